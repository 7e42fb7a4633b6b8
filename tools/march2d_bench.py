"""Back-to-back MatMult on 2D box stencils: the z-march (default) against the row-parallel ELL kernel
(MSPLIT_TUNING 268435456), HIP-event timing of the library, bitwise check.  Prints one JSON object."""
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch  # noqa: F401
    from medane_tchakorom_ufc_thesis_repository_amd import _lib
    from medane_tchakorom_ufc_thesis_repository_amd.petsc import Context, Mat, Vec
    L = _lib.load()
    L.msk_set_tuning.argtypes = [ctypes.c_int]
    ctx = Context(0)
    out = {}
    for nx, ny in ((4096, 4096), (8192, 8192), (2000, 3000)):
        A = Mat.box_stencil(ctx, 2, nx, ny)
        n = nx * ny
        x = Vec.from_array(ctx, np.random.default_rng(1).uniform(-1, 1, n))
        y = Vec(ctx, n)
        res, ys = {}, {}
        for r in range(3):
            for t in (0, 268435456):
                L.msk_set_tuning(t)
                ctx.reset_kernel_stats()
                ctx.set_timing(True)
                for _ in range(20):
                    A.mult(x, y)
                ctx.set_timing(False)
                s = ctx.kernel_stats()["spmv"]
                res.setdefault(t, []).append(s["ms"] / s["launches"] * 1e3)
                ys[t] = y.get_array()
        L.msk_set_tuning(0)
        out[f"{nx}x{ny}"] = {"march_us": float(np.median(res[0])), "rowpar_us": float(np.median(res[268435456])),
                             "bitwise": bool(np.array_equal(ys[0], ys[268435456]))}
        del A, x, y
    print(json.dumps(out))


if __name__ == "__main__":
    main()
