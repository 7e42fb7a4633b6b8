"""Measurement of the asynchronous rows on one GPU.

1. Transport: the newest-value slots (msp_amsg, a boundary plane) and the
   R-row broadcast (msp_abcast, a dense block), GB/s of payload per send +
   receive pair, both ends in this process: host-staged (HBM -> shared memory
   -> HBM) and through HBM slots (on one GPU a same-device copy; between GPUs
   the receive is a peer copy over xGMI).
2. AM / AMAM-global on nb z-slab blocks of one GPU, round-robin (LocalComm):
   DOF-updates/s of the inner GMRES and the share of host time in each phase
   (solve, exchange, minimize, detect).

  python tools/async_bench.py [--n 256] [--planes 128] [--nb 2] [--variant am]
         [--inner-max-it 20] [--max-iterations 60] [--s 4]
Prints one JSON object.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
import uuid

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def transport(ctx, n_plane: int, rows: int, s: int, reps: int, modes=("host", "device")):
    """Payload GB/s of one send + receive, host-staged and through HBM slots."""
    from medane_tchakorom_ufc_thesis_repository_amd.petsc import AsyncBroadcast, AsyncMessages, DenseMat, Vec
    import numpy as np
    out = {}
    x = Vec.from_array(ctx, np.arange(n_plane, dtype=np.float64))
    y = Vec(ctx, n_plane)
    R = DenseMat(ctx, rows, s)
    for j in range(s):
        R.set_column(j, 0, Vec.from_array(ctx, np.full(rows, float(j))))
    R2 = DenseMat(ctx, rows, s)
    for mode in modes:
        name = f"/msplit_tb_{os.getpid()}_{uuid.uuid4().hex[:8]}"
        a = AsyncMessages(name, 2, 0, n_plane, owner=True)
        b = AsyncMessages(name, 2, 1, n_plane, owner=False)
        if mode == "device":
            a.enable_device(ctx)
            b.enable_device(ctx)
        a.send_vec(1, [0, 0], x, 0, n_plane)
        b.recv_vec(0, 2, y, 0, n_plane)                   # first use: registration / IPC resolution
        ctx.synchronize()
        t0 = time.perf_counter()
        for k in range(reps):
            a.send_vec(1, [0, k + 1], x, 0, n_plane)
            got, _, _ = b.recv_vec(0, 2, y, 0, n_plane)
            assert got
        host = (time.perf_counter() - t0) / reps      # what the caller's thread spends per pair
        ctx.synchronize()                             # device slots: the copies complete on the stream
        dt = (time.perf_counter() - t0) / reps
        out[f"amsg_plane_{mode}"] = {"doubles": n_plane, "us_per_send_recv": dt * 1e6,
                                     "host_us_per_send_recv": host * 1e6, "GBps": 8 * n_plane / dt / 1e9}
        b.close_peers()
        a.close_peers()
        b.destroy()
        a.destroy()
        name = f"/msplit_tb_{os.getpid()}_{uuid.uuid4().hex[:8]}"
        p = AsyncBroadcast(name, 2, 0, rows * s, owner=True)
        q = AsyncBroadcast(name, 2, 1, rows * s, owner=False)
        if mode == "device":
            p.enable_device(ctx)
            q.enable_device(ctx)
        p.publish_dense(R)
        q.fetch_dense(0, R2)
        nrep = max(2, reps // 10)
        t0 = time.perf_counter()
        for _ in range(nrep):
            assert p.publish_dense(R)
            assert q.fetch_dense(0, R2)
        dt = (time.perf_counter() - t0) / nrep
        out[f"abcast_R_{mode}"] = {"rows": rows, "cols": s, "ms_per_publish_fetch": dt * 1e3,
                                   "GBps": 8 * rows * s / dt / 1e9}
        q.close_peers()
        p.close_peers()
        q.destroy()
        p.destroy()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=256, help="nx = ny")
    ap.add_argument("--planes", type=int, default=128, help="z-planes per block")
    ap.add_argument("--nb", type=int, default=2)
    ap.add_argument("--variant", default="am", choices=["am", "amam_global"])
    ap.add_argument("--inner-max-it", type=int, default=20)
    ap.add_argument("--max-iterations", type=int, default=60)
    ap.add_argument("--s", type=int, default=4)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--rtol", type=float, default=1e-6)
    ap.add_argument("--transport", default="device", choices=["device", "host"])
    ap.add_argument("--transport-modes", default="host,device", help="modes of the transport measurement")
    ap.add_argument("--transport-only", action="store_true", help="measure the transport, skip the solve")
    args = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime)
    from medane_tchakorom_ufc_thesis_repository_amd.asynchronous import am_solve
    from medane_tchakorom_ufc_thesis_repository_amd.comm import LocalComm
    from medane_tchakorom_ufc_thesis_repository_amd.multisplitting import make_blocks
    from medane_tchakorom_ufc_thesis_repository_amd.petsc import Context, Options

    ctx = Context(0)
    n, nb = args.n, args.nb
    rows = n * n * args.planes
    out = {"transport": transport(ctx, n * n, rows, args.s, args.reps, tuple(args.transport_modes.split(",")))}
    if args.transport_only:
        print(json.dumps(out, indent=1))
        return
    inner = " ".join(f"-inner{b + 1}_ksp_max_it {args.inner_max_it} -inner{b + 1}_ksp_rtol 1e-20 "
                     f"-inner{b + 1}_pc_type none" for b in range(nb))
    outer = " ".join(f"-outer{b + 1}_ksp_type lsqr -outer{b + 1}_ksp_convergence_test default "
                     f"-outer{b + 1}_ksp_lsqr_exact_mat_norm -outer{b + 1}_ksp_atol 1e-100 "
                     f"-outer{b + 1}_ksp_max_it 70 -outer{b + 1}_ksp_rtol 1e-15" for b in range(nb))
    opts = Options(inner + " " + outer)
    comm = LocalComm()
    blocks = make_blocks(ctx, 3, n, n, args.planes * nb, nb, range(nb), opts, comm)
    if args.variant == "amam_global":
        for blk in blocks:
            blk.setup_global_async_minimization(args.s)
    ctx.synchronize()
    res = am_solve(blocks, comm, rtol=args.rtol, max_iterations=args.max_iterations, variant=args.variant,
                   s=args.s, stop_at_limit=True, transport=args.transport)
    inner_total = sum(res.inner_its)
    tot = sum(res.timers.values())
    out["solve"] = {"variant": args.variant, "transport": res.transport, "mesh": [n, n, args.planes * nb],
                    "blocks": nb, "rows_per_block": rows, "iterations": res.iterations, "inner_its": res.inner_its,
                    "converged": res.converged, "final_norm_rel": res.final_norm / res.norm0,
                    "elapsed_s": res.elapsed, "DOF_updates_per_s": rows * inner_total / res.elapsed,
                    "phase_share": {k: v / tot for k, v in res.timers.items()} if tot else {},
                    "phase_s": res.timers}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
