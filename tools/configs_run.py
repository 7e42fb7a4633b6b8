"""Solve BASELINE.json's configurations end to end on one MI355X.

  c1: configs[0] -- 2D 5-pt Poisson 256x256, SMSM-global, 2 blocks, the
      campaign options (default_run_variables:34-52, running_bulk_test_g5k:
      247-248): -s 4 -rtol 1e-3, inner GMRES(30) max_it 20 rtol 1e-3, outer
      LSQR max_it 70 rtol 1e-15 exact norm.  Solved to convergence on the GPU
      and by the CPU oracle in PETSc (sequential) order and in the GPU's (DBR)
      order; the GPU run must equal the DBR oracle bit for bit.
  c3: configs[2] -- 3D 7-pt Poisson 512^3, SMSM-global, 2 blocks, s = 20 (both
      blocks on this one GPU, round-robin), up to --max-outer outer iterations.
  c5: configs[4] -- 3D convection-diffusion 512^3, AMAM-global, 2 blocks on this
      GPU (round-robin, HBM mailboxes), up to --max-outer outer iterations.

Prints one JSON object per configuration.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _opts(nb, inner_max_it, inner_rtol, s):
    from medane_tchakorom_ufc_thesis_repository_amd.petsc import Options
    inner = " ".join(f"-inner{b + 1}_ksp_type gmres -inner{b + 1}_ksp_gmres_restart 30 -inner{b + 1}_ksp_max_it "
                     f"{inner_max_it} -inner{b + 1}_ksp_rtol {inner_rtol} -inner{b + 1}_pc_type none "
                     f"-inner{b + 1}_ksp_norm_type unpreconditioned" for b in range(nb))
    outer = " ".join(f"-outer{b + 1}_ksp_type lsqr -outer{b + 1}_ksp_convergence_test default "
                     f"-outer{b + 1}_ksp_lsqr_exact_mat_norm -outer{b + 1}_ksp_atol 1e-100 "
                     f"-outer{b + 1}_ksp_max_it 70 -outer{b + 1}_ksp_rtol 1e-15 -outer{b + 1}_pc_type none"
                     for b in range(nb))
    return Options(f"{inner} {outer} -s {s}")


def run_c1(ctx, args):
    import numpy as np
    from medane_tchakorom_ufc_thesis_repository_amd.comm import LocalComm
    from medane_tchakorom_ufc_thesis_repository_amd.multisplitting import make_smsm, smsm_solve
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as po
    m = n = 256
    nb, s, rtol, irtol = 2, 4, 1e-3, 1e-3
    comm = LocalComm()
    blocks, mini = make_smsm(ctx, 2, m, n, 1, nb, range(nb), s, _opts(nb, 20, irtol, s), comm)
    ctx.synchronize()
    t0 = time.perf_counter()
    res = smsm_solve(blocks, comm, s, mini, rtol=rtol, max_outer=1000)
    ctx.synchronize()
    t_gpu = time.perf_counter() - t0
    inner = dict(restart=30, max_it=20, rtol=irtol, abstol=1e-50)
    outer = dict(max_it=70, rtol=1e-15, abstol=1e-100, exact_norm=1, conv_test=0)
    out = {"config": "c1: 2D 5-pt Poisson 256x256, SMSM-global, 2 blocks, s 4, rtol 1e-3 (configs[0])",
           "gpu": {"outer_its": res.outer_its, "seconds": t_gpu, "final_norm": res.final_norm, "error": res.error,
                   "inner_its_total": int(np.sum(res.inner_its)), "hist": res.hist}}
    for name, mode in (("oracle_dbr", po.REDUCE_DBR), ("oracle_petsc_order", po.REDUCE_SEQ)):
        t0 = time.perf_counter()
        ro = po.smsm_solve(2, m, n, 1, nb, s, rtol, dict(inner, reduce_mode=mode), dict(outer, reduce_mode=mode),
                           max_outer=1000)
        dt = time.perf_counter() - t0
        out[name] = {"outer_its": ro["outer_its"], "seconds": dt, "final_norm": ro["final_norm"],
                     "error": ro["error"], "hist": ro["hist"].tolist()}
        if mode == po.REDUCE_DBR:
            x = np.concatenate([blk.x.get_array() for blk in blocks])
            out["bitwise_vs_dbr_oracle"] = bool(res.outer_its == ro["outer_its"] and
                                                np.array_equal(np.array(res.hist), ro["hist"]) and
                                                np.array_equal(x, ro["x"]))
    out["cpu_cores"] = 1
    return out


def run_c3(ctx, args):
    import numpy as np
    from medane_tchakorom_ufc_thesis_repository_amd.comm import LocalComm
    from medane_tchakorom_ufc_thesis_repository_amd.multisplitting import make_smsm, smsm_solve
    n, nb, s = args.n, 2, 20
    comm = LocalComm()
    blocks, mini = make_smsm(ctx, 3, n, n, n, nb, range(nb), s, _opts(nb, 20, 1e-20, s), comm)
    ctx.synchronize()
    t0 = time.perf_counter()
    res = smsm_solve(blocks, comm, s, mini, rtol=1e-4, max_outer=args.max_outer)
    ctx.synchronize()
    dt = time.perf_counter() - t0
    rows = n * n * n
    its = int(np.sum(res.inner_its))
    return {"config": f"c3: 3D 7-pt Poisson {n}^3, SMSM-global, 2 blocks on one GPU, s 20, rtol 1e-4 (configs[2])",
            "outer_its": res.outer_its, "converged": bool(res.hist and res.hist[-1] <= 1e-4 * res.norm0),
            "seconds": dt, "seconds_per_outer": dt / max(res.outer_its, 1),
            "DOF_updates_per_s": rows // nb * its / dt, "hist_rel": [h / res.norm0 for h in res.hist],
            "lsqr_its": res.lsqr_its, "final_norm_rel": res.final_norm / res.norm0, "error": res.error}


def run_c5(ctx, args):
    from medane_tchakorom_ufc_thesis_repository_amd.asynchronous import am_solve
    from medane_tchakorom_ufc_thesis_repository_amd.comm import LocalComm
    from medane_tchakorom_ufc_thesis_repository_amd.multisplitting import make_blocks
    n, nb, s = args.n, 2, 20
    pe = tuple(float(v) for v in args.peclet.split(","))
    comm = LocalComm()
    blocks = make_blocks(ctx, 3, n, n, n, nb, range(nb), _opts(nb, 20, 1e-20, s), comm, pe)
    for blk in blocks:
        blk.setup_global_async_minimization(s)
    ctx.synchronize()
    res = am_solve(blocks, comm, rtol=1e-4, max_iterations=args.max_outer, variant="amam_global", s=s,
                   stop_at_limit=True)
    rows = n * n * n
    return {"config": f"c5: 3D convection-diffusion {n}^3 (cell Peclet {pe}), AMAM-global, 2 blocks on one GPU, "
                      f"s 20 (configs[4] algorithm)", "transport": res.transport,
            "iterations": res.iterations, "converged": res.converged, "seconds": res.elapsed,
            "DOF_updates_per_s": rows // nb * sum(res.inner_its) / res.elapsed,
            "final_norm_rel": res.final_norm / res.norm0, "error": res.error,
            "phase_share": {k: v / sum(res.timers.values()) for k, v in res.timers.items()}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c1")
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--max-outer", type=int, default=10)
    ap.add_argument("--peclet", default="0.5,0.25,-0.3")
    args = ap.parse_args()
    import torch  # noqa: F401
    from medane_tchakorom_ufc_thesis_repository_amd.petsc import Context
    ctx = Context(0)
    for c in args.configs.split(","):
        out = {"c1": run_c1, "c3": run_c3, "c5": run_c5}[c](ctx, args)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
