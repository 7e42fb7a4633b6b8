"""AMAM-global (configs[3] / configs[4]'s algorithm) at the real per-GPU block size on one MI355X.

  pair       two blocks of the configs[3] geometry (1024 x 1024 x 128 each, Poisson) or, with --peclet,
             of configs[4] (512 x 512 x 64, upwind convection-diffusion), round-robin on this GPU
             (LocalComm, HBM mailboxes): per-iteration local norms, phase timers and peak HBM, for the
             replicated-R LSQR (outer_solver_norm_equation, utils.c:1061-1078) and for the reference's
             normal-equations step (outer_solver, utils.c:972-996: -msplit_minimization rtr).
  footprint  one interior rank of the 8-block configs[3] run (1024^3 / 8): its real block, and for "lsqr"
             the replicated R of all 8 row blocks (7 peer blocks filled on the device from its own rows),
             the global b, the broadcast buffers with nbuf chosen by the production free-HBM rule; one
             full outer iteration (s inner solves, R = A S, publish, the 8-row-block LSQR, x = S alpha).
             For "rtr" the same rank with 8 Gram parts instead.  Peak HBM (device-wide, sampled) and the
             minimization time.

  whole      all 8 blocks of configs[4] (--n 512 --peclet ...; or configs[3] geometry at --n) round-robin on this
             GPU, each with its replicated R, global b and broadcast buffers: HBM marks after the blocks, after the
             minimization setup, and the peak over --its outer iterations per block (stop_at_limit), or the
             allocation that failed.

  python tools/amam_configs.py pair [--peclet 0.5,0.25,-0.3] [--its 2] [--minimization lsqr,rtr]
  python tools/amam_configs.py whole --n 512 --peclet 0.5,0.25,-0.3 --its 1 [--minimization lsqr]
  python tools/amam_configs.py footprint [--minimization lsqr|rtr]
Prints one JSON object per measurement.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time
import uuid

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


class HbmSampler:
    """Device-wide HBM in use (hipMemGetInfo, which sees the library's own hipMalloc'd memory as well as
    torch's), sampled every 20 ms on a thread: the peak over the run."""

    def __init__(self, dev=0):
        import torch
        self.torch, self.dev = torch, dev
        free, self.total = torch.cuda.mem_get_info(dev)
        self.base = self.total - free
        self.peak = self.base
        self._stop = False
        self.t = threading.Thread(target=self._run, daemon=True)
        self.t.start()

    def used(self):
        free, _ = self.torch.cuda.mem_get_info(self.dev)
        return self.total - free

    def _run(self):
        while not self._stop:
            self.peak = max(self.peak, self.used())
            time.sleep(0.02)

    def stop(self):
        self._stop = True
        self.t.join()
        self.peak = max(self.peak, self.used())
        return {"peak_GB": self.peak / 1e9, "total_GB": self.total / 1e9, "before_GB": self.base / 1e9}


def options(nb, s, inner_max_it, minimization):
    return " ".join(
        f"-inner{b + 1}_ksp_type gmres -inner{b + 1}_ksp_gmres_restart 30 -inner{b + 1}_ksp_max_it {inner_max_it} "
        f"-inner{b + 1}_ksp_rtol 1e-20 -inner{b + 1}_ksp_atol 1e-100 -inner{b + 1}_pc_type none "
        f"-outer{b + 1}_ksp_type lsqr -outer{b + 1}_ksp_convergence_test default -outer{b + 1}_ksp_lsqr_exact_mat_norm "
        f"-outer{b + 1}_ksp_atol 1e-100 -outer{b + 1}_ksp_max_it 70 -outer{b + 1}_ksp_rtol 1e-15 "
        f"-outer{b + 1}_pc_type none" for b in range(nb)) + f" -s {s} -msplit_minimization {minimization}"


def pair(args, minimization):
    import torch
    from medane_tchakorom_ufc_thesis_repository_amd.asynchronous import am_solve
    from medane_tchakorom_ufc_thesis_repository_amd.comm import LocalComm
    from medane_tchakorom_ufc_thesis_repository_amd.multisplitting import make_blocks
    from medane_tchakorom_ufc_thesis_repository_amd.petsc import Context, Options
    n, planes = (512, 64) if args.peclet else (1024, 128)
    ctx = Context(0)
    hbm = HbmSampler()
    t0 = time.perf_counter()
    opts = Options(options(2, args.s, args.inner_max_it, minimization))
    comm = LocalComm()
    blocks = make_blocks(ctx, 3, n, n, 2 * planes, 2, [0, 1], opts, comm, args.peclet)
    for blk in blocks:
        blk.setup_global_async_minimization(args.s)
    ctx.synchronize()
    setup_s = time.perf_counter() - t0
    res = am_solve(blocks, comm, rtol=args.rtol, record=True, variant="amam_global", s=args.s,
                   max_iterations=args.its, stop_at_limit=True)
    torch.cuda.synchronize()
    mem = hbm.stop()
    rows = n * n * planes
    return {"mode": "pair", "minimization": minimization,
            "geometry": f"2 blocks of {n}x{n}x{planes} ({'configs[4] convection-diffusion' if args.peclet else 'configs[3] Poisson'}), round-robin on one GPU",
            "s": args.s, "inner_max_it": args.inner_max_it, "iterations": res.iterations, "inner_its": res.inner_its,
            "converged": res.converged, "norm0": res.norm0, "final_norm": res.final_norm,
            "trace": [(b, it, ln) for b, it, ln, _, _ in res.trace], "elapsed_s": res.elapsed, "setup_s": setup_s,
            "timers_s": res.timers, "dof_updates_per_s": rows * sum(res.inner_its) / res.elapsed, "hbm": mem,
            "transport": res.transport}


def footprint(args, minimization):
    import torch
    from medane_tchakorom_ufc_thesis_repository_amd.comm import LocalComm
    from medane_tchakorom_ufc_thesis_repository_amd.multisplitting import GpuBlock
    from medane_tchakorom_ufc_thesis_repository_amd.petsc import AsyncBroadcast, Context, DenseMat, Options
    from medane_tchakorom_ufc_thesis_repository_amd.utils import block_layout
    nb, rank, n = 8, 3, 1024
    ctx = Context(0)
    hbm = HbmSampler()
    marks = {}
    t0 = time.perf_counter()
    opts = Options(options(nb, args.s, args.inner_max_it, minimization))
    L = block_layout(3, n, n, n, nb, rank, None)
    blk = GpuBlock(ctx, L, opts, LocalComm())
    blk.setup_global_async_minimization(args.s)
    ctx.synchronize()
    marks["after_setup_GB"] = hbm.used() / 1e9
    name = f"/msplit_fp_{os.getpid()}_{uuid.uuid4().hex[:8]}"
    bc = AsyncBroadcast(name + "_R", nb, rank, blk.bcast_cap(), True)
    nbuf = int(os.environ.get("MSPLIT_ABCAST_NBUF", "0"))
    # the production rule (asynchronous.AsyncBlock.enable_device -> msp_abcast_enable_device with nbuf 0)
    nbuf = bc.enable_device(ctx, nbuf if nbuf in (1, 2) else 0)
    ctx.synchronize()
    marks["after_broadcast_buffers_GB"] = hbm.used() / 1e9
    blk.reset_halo()
    tim = {}
    t1 = time.perf_counter()
    its = 0
    for k in range(args.s):                          # AMAM-global_prime.c:378-413 (no peers: the halo stays 0)
        blk.update_rhs()
        its += blk.solve()
        blk.store_column(k)
    ctx.synchronize()
    tim["inner_s"] = time.perf_counter() - t1
    if minimization == "lsqr":                       # the 7 peer blocks' rows of R: this block's own R, on the device
        blk.form_R()
        for j, R in enumerate(blk.R_rep):
            if j != rank:
                for c in range(args.s):
                    R.set_column(c, 0, blk.R.column_vec(c))
    else:                                            # 7 peer Gram parts: this block's own part
        blk.form_R()
        blk.R.gram(blk.b, blk.Gc)
        for j, G in enumerate(blk.Gc_rep):
            if j != rank:
                for c in range(args.s + 1):
                    G.set_column(c, 0, blk.Gc.column_vec(c))
    ctx.synchronize()
    marks["after_peer_fill_GB"] = hbm.used() / 1e9
    t2 = time.perf_counter()
    rn, lits, reason = blk.global_async_minimize(bc)   # form_R, publish, fetch (none newer), LSQR, x = S alpha
    ctx.synchronize()
    tim["minimize_s"] = time.perf_counter() - t2
    mem = hbm.stop()
    bc.close_peers()
    bc.destroy()
    return {"mode": "footprint", "minimization": minimization,
            "rank": f"block {rank} of {nb} of 1024^3 (1024x1024x128 rows, both halos)", "s": args.s,
            "nbuf": nbuf, "inner_gmres_its": its, "lsqr_its": lits, "lsqr_reason": reason, "lsqr_rnorm": rn,
            "times": tim, "hbm": mem, "hbm_marks": marks, "setup_s": t1 - t0,
            "replicated_R_GB": (8 * L.nrows * args.s * 8 / 1e9) if minimization == "lsqr" else 8 * args.s * (args.s + 1) * 8 / 1e9}


def whole(args, minimization):
    import torch
    from medane_tchakorom_ufc_thesis_repository_amd.asynchronous import am_solve
    from medane_tchakorom_ufc_thesis_repository_amd.comm import LocalComm
    from medane_tchakorom_ufc_thesis_repository_amd.multisplitting import make_blocks
    from medane_tchakorom_ufc_thesis_repository_amd.petsc import Context, Options
    nb, n = 8, args.n
    ctx = Context(0)
    hbm = HbmSampler()
    marks, t0 = {}, time.perf_counter()
    out = {"mode": "whole", "minimization": minimization, "geometry": f"{n}^3 in {nb} blocks of {n}x{n}x{n // nb}",
           "peclet": args.peclet, "s": args.s, "inner_max_it": args.inner_max_it,
           "nbuf_env": os.environ.get("MSPLIT_ABCAST_NBUF", "0")}
    stage = "blocks"
    try:
        comm = LocalComm()
        blocks = make_blocks(ctx, 3, n, n, n, nb, range(nb), Options(options(nb, args.s, args.inner_max_it,
                                                                            minimization)), comm, args.peclet)
        ctx.synchronize()
        marks["after_blocks_GB"] = hbm.used() / 1e9
        stage = "minimization setup"
        for blk in blocks:
            blk.setup_global_async_minimization(args.s)
        ctx.synchronize()
        marks["after_minimization_setup_GB"] = hbm.used() / 1e9
        stage = "run"
        res = am_solve(blocks, comm, rtol=args.rtol, variant="amam_global", s=args.s, max_iterations=args.its,
                       stop_at_limit=True)
        torch.cuda.synchronize()
        out.update({"iterations": res.iterations, "inner_its": res.inner_its, "elapsed_s": res.elapsed,
                    "timers_s": res.timers, "final_norm": res.final_norm, "norm0": res.norm0, "ok": True})
    except Exception as e:                            # an allocation that does not fit: say which stage
        out.update({"ok": False, "failed_stage": stage, "error": str(e)[:300]})
    out.update({"hbm": hbm.stop(), "hbm_marks": marks, "wall_s": time.perf_counter() - t0})
    return out


def main():
    p = argparse.ArgumentParser()
    p.add_argument("mode", choices=["pair", "footprint", "whole"])
    p.add_argument("--n", type=int, default=512)
    p.add_argument("--minimization", default="lsqr,rtr")
    p.add_argument("--peclet", default=None)
    p.add_argument("--its", type=int, default=2)
    p.add_argument("--s", type=int, default=20)
    p.add_argument("--inner-max-it", type=int, default=20)
    p.add_argument("--rtol", type=float, default=1e-30)
    a = p.parse_args()
    a.peclet = tuple(float(v) for v in a.peclet.split(",")) if a.peclet else None
    import torch
    torch.cuda.set_device(0)
    for m in a.minimization.split(","):
        out = pair(a, m) if a.mode == "pair" else footprint(a, m) if a.mode == "footprint" else whole(a, m)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
