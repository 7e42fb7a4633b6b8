"""Per-kernel HBM bandwidth of the hot-path kernels on 256^3-sized operands.

Times each kernel class with the library's HIP-event timing, interleaving
kernel variants (msk_set_variant) in one process so A/B deltas are not
cross-process noise.  Prints one JSON object.

  python tools/microbench.py [--n 256] [--reps 20] [--rounds 3]
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
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", default="spmv:0;maxpy:0,1;mdot:0")
    args = ap.parse_args()
    import numpy as np
    import torch  # noqa: F401
    from medane_tchakorom_ufc_thesis_repository_amd import _lib
    from medane_tchakorom_ufc_thesis_repository_amd.petsc import Context, Mat, Vec
    L = _lib.load()
    L.msk_set_variant.argtypes = [ctypes.c_int, ctypes.c_int]
    L.msk_set_variant.restype = None
    which = {"spmv": 0, "mdot": 1, "maxpy": 2}

    n = args.n
    N = n ** 3
    ctx = Context(0)
    A = Mat.box_stencil(ctx, 3, n, n, n)
    rng = np.random.default_rng(1)
    V = [Vec.from_array(ctx, rng.uniform(-1, 1, N)) for _ in range(31)]
    w = Vec.from_array(ctx, rng.uniform(-1, 1, N))
    y = Vec(ctx, N)

    def timed(fn, cls):
        ctx.reset_kernel_stats()
        ctx.set_timing(True)
        for _ in range(args.reps):
            fn()
        ctx.set_timing(False)
        s = ctx.kernel_stats()[cls]
        return s["bytes"] / (s["ms"] * 1e-3) / 1e9, s["ms"] / s["launches"] * 1e3

    res = {}
    variants = {}
    for item in args.variants.split(";"):
        k, vs = item.split(":")
        variants[k] = [int(v) for v in vs.split(",")]
    for rnd in range(args.rounds):
        for v in variants.get("spmv", [0]):
            L.msk_set_variant(which["spmv"], v)
            gb, us = timed(lambda: A.mult(w, y), "spmv")
            res.setdefault(f"spmv/v{v}", []).append((gb, us))
        for v in variants.get("mdot", [0]):
            L.msk_set_variant(which["mdot"], v)
            for k in (1, 8, 16, 30):
                gb, us = timed(lambda: w.mdot(V[:k]), "mdot")
                res.setdefault(f"mdot{k}/v{v}", []).append((gb, us))
        for v in variants.get("maxpy", [0]):
            L.msk_set_variant(which["maxpy"], v)
            for k in (1, 8, 16, 30):
                a = np.full(k, 1e-300)
                gb, us = timed(lambda: w.maxpy(a, V[:k]), "maxpy")
                res.setdefault(f"maxpy{k}/v{v}", []).append((gb, us))
        gb, us = timed(lambda: w.norm(), "norm")
        res.setdefault("norm", []).append((gb, us))
        gb, us = timed(lambda: w.scale(1.0000000001), "scale")
        res.setdefault("scale", []).append((gb, us))
    out = {k: {"GBps_median": float(np.median([g for g, _ in v])), "GBps_max": float(max(g for g, _ in v)),
               "us_median": float(np.median([u for _, u in v]))} for k, v in res.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
