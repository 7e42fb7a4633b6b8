"""Per-kernel HBM bandwidth of the hot-path kernels.

Times each kernel class with the library's HIP-event timing, interleaving
tuning settings (msk_set_tuning flags, msk_set_spmv_group) in one process so
A/B deltas are not cross-process noise.  Prints one JSON object.

  python tools/microbench.py [--n 256] [--nz 256] [--reps 20] [--rounds 3]
         [--tunings 0,4] [--groups 0] [--kernels spmv,mdot,maxpy,lsqr]
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
    ap.add_argument("--n", type=int, default=256, help="nx = ny")
    ap.add_argument("--nz", type=int, default=None)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--tunings", default="0")
    ap.add_argument("--groups", default="0", help="SpMV XCD group sizes to sweep (0 = auto)")
    ap.add_argument("--march-z", default="0", help="z-march planes per workgroup to sweep (0 = auto)")
    ap.add_argument("--march-lines", default="0", help="z-march tiles to sweep (1 = 256 plane rows, 4 = 4 lines)")
    ap.add_argument("--kernels", default="spmv,mdot,maxpy")
    ap.add_argument("--storage", default="csr", choices=["csr", "dv"], help="SpMV entry storage")
    args = ap.parse_args()
    import numpy as np
    import torch  # noqa: F401
    from medane_tchakorom_ufc_thesis_repository_amd import _lib
    from medane_tchakorom_ufc_thesis_repository_amd.petsc import LSQR, Context, DenseMat, Mat, Vec
    L = _lib.load()
    L.msk_set_tuning.argtypes = [ctypes.c_int]
    L.msk_set_tuning.restype = None
    L.msk_set_spmv_group.argtypes = [ctypes.c_int]
    L.msk_set_spmv_group.restype = None
    L.msk_set_march_z.argtypes = [ctypes.c_int]
    L.msk_set_march_z.restype = None
    L.msk_set_march_lines.argtypes = [ctypes.c_int]
    L.msk_set_march_lines.restype = None
    zs = [(int(z), int(m)) for z in args.march_z.split(",") for m in args.march_lines.split(",")]
    kernels = args.kernels.split(",")
    tunings = [int(t) for t in args.tunings.split(",")]
    groups = [int(g) for g in args.groups.split(",")]

    n = args.n
    nz = args.nz or n
    N = n * n * nz
    ctx = Context(0)
    A = Mat.box_stencil(ctx, 3, n, n, nz)
    A.set_storage(args.storage)
    rng = np.random.default_rng(1)
    w = Vec.from_array(ctx, rng.uniform(-1, 1, N))
    y = Vec(ctx, N)
    V = [Vec.from_array(ctx, rng.uniform(-1, 1, N)) for _ in range(31)] if ("mdot" in kernels or "maxpy" in kernels) else []
    if "lsqr" in kernels:
        s = 20
        R = DenseMat(ctx, N, s)
        for j in range(s):    # independent columns, so the LSQR runs its max_it steps
            R.set_column(j, 0, Vec.from_array(ctx, rng.uniform(-1, 1, N)))
        l = LSQR(ctx)
        l._set(max_it=70, rtol=1e-15, abstol=1e-100, exact_norm=1, conv_test=0)
        l.set_operators([R])
        alpha = Vec(ctx, s)

    def timed(fn, cls):
        ctx.reset_kernel_stats()
        ctx.set_timing(True)
        for _ in range(args.reps):
            fn()
        ctx.set_timing(False)
        st = ctx.kernel_stats()
        s = st[cls]
        return s["bytes"] / (s["ms"] * 1e-3) / 1e9, s["ms"] / max(s["launches"], 1) * 1e3

    res = {}
    y_ref, mismatch = None, []
    for _ in range(args.rounds):
        for t in tunings:
            L.msk_set_tuning(t)
            for g in (groups if "spmv" in kernels else [0]):
                L.msk_set_spmv_group(g)
                for z, ml in (zs if "spmv" in kernels else [(0, 0)]):
                    L.msk_set_march_z(z)
                    L.msk_set_march_lines(ml)
                    if "spmv" in kernels:
                        key = f"spmv/t{t}/g{g}" + (f"/z{z}/l{ml}" if len(zs) > 1 else "")
                        gb, us = timed(lambda: A.mult(w, y), "spmv")
                        res.setdefault(key, []).append((gb, us))
                        ya = y.get_array()
                        if y_ref is None:
                            y_ref = ya
                        elif not np.array_equal(ya, y_ref):
                            mismatch.append(key)
                L.msk_set_march_z(0)
                L.msk_set_march_lines(0)
            L.msk_set_spmv_group(0)
            if "mdot" in kernels:
                for k in (1, 2, 4, 8, 12, 16, 20, 30):
                    gb, us = timed(lambda: w.mdot(V[:k]), "mdot")
                    res.setdefault(f"mdot{k}/t{t}", []).append((gb, us))
            if "maxpy" in kernels:
                for k in (1, 2, 4, 8, 12, 16, 20, 30):
                    a = np.full(k, 1e-300)
                    gb, us = timed(lambda: w.maxpy(a, V[:k]), "maxpy")
                    res.setdefault(f"maxpy{k}/t{t}", []).append((gb, us))
            if "lsqr" in kernels:
                for cls in ("dgemv", "dgemvt"):
                    gb, us = timed(lambda: l.solve([w], alpha), cls)
                    res.setdefault(f"lsqr_{cls}/t{t}", []).append((gb, us))
    L.msk_set_tuning(0)
    out = {k: {"GBps_median": float(np.median([g for g, _ in v])), "GBps_max": float(max(g for g, _ in v)),
               "us_median": float(np.median([u for _, u in v]))} for k, v in res.items()}
    out["spmv_bitwise_equal_across_tunings"] = not mismatch
    out["spmv_mismatch"] = sorted(set(mismatch))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
