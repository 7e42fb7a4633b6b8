"""Same-process A/B of the CSR MatMult cache policy on the 512^3 7-point matrix:
the default policy (flags 0) against non-temporal col/val loads and y stores
(MSK_TUNE_SPMV_TEMPORAL = 2 since round 2; before it, 2 selected non-temporal), interleaved, timed with the library's per-launch HIP
events.

  python tools/spmv_policy_ab.py [--n 512] [--reps 10] [--rounds 5]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--flags", default="0,2")
    ap.add_argument("--no-torch", action="store_true", help="library stream only (no torch in the process)")
    ap.add_argument("--own-stream", action="store_true", help="torch imported, but the library's own stream")
    ap.add_argument("--lib-first", action="store_true",
                    help="load the library (and so /opt/rocm's HIP runtime) before importing torch")
    args = ap.parse_args()
    import numpy as np
    if args.lib_first:
        from medane_tchakorom_ufc_thesis_repository_amd import _lib as _l0
        _l0.load()
    if args.no_torch:
        torch = None
    else:
        import torch
    from medane_tchakorom_ufc_thesis_repository_amd import _lib
    from medane_tchakorom_ufc_thesis_repository_amd.petsc import Context, Mat, Vec
    L = _lib.load()
    L.msk_set_tuning.argtypes = [ctypes.c_int]
    L.msk_set_tuning.restype = None
    stream = torch.cuda.current_stream() if torch and not args.own_stream else None
    ctx = Context(0, stream=stream.cuda_stream) if stream is not None else Context(0)
    n = args.n
    A = Mat.box_stencil(ctx, 3, n, n, n)
    A.set_storage("csr")
    N = A.shape[0]
    alg = 12.0 * A.nnz + 20.0 * N + 4.0
    x = Vec.from_array(ctx, np.random.default_rng(20251121).uniform(-1, 1, N))
    y = Vec(ctx, N)
    flags = [int(f) for f in args.flags.split(",")]
    res = {f: {"event_us": []} for f in flags}
    for _ in range(args.rounds):
        for f in flags:
            L.msk_set_tuning(f)
            A.mult(x, y)
            ctx.set_timing(True, 1)
            ctx.reset_kernel_stats()
            for _ in range(args.reps):
                A.mult(x, y)
            st = ctx.kernel_stats()["spmv"]
            ctx.set_timing(False)
            res[f]["event_us"].append(st["ms"] / st["launches"] * 1e3)
    L.msk_set_tuning(0)
    out = {}
    for f, r in res.items():
        out[str(f)] = {k: {"median_us": float(np.median(v)), "frac": alg / (np.median(v) * 1e-6) / 8e12}
                       for k, v in r.items()}
    maps = open("/proc/self/maps").read().split("\n")
    out["_runtime"] = sorted({ln.split()[-1] for ln in maps if "libamdhip64" in ln})
    out["_stream"] = None if stream is None else int(stream.cuda_stream)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
