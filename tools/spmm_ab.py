"""R = A_ext S (MatMatMult, DV storage) on one SMSM block, for the MSPLIT_SPMM_COLS A/B (one process per value).

  MSPLIT_SPMM_COLS=4 python tools/spmm_ab.py [--n 512] [--planes 256] [--s 20]
Prints the per-launch time (HIP events) and a hash of R (bitwise comparison across values)."""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--planes", type=int, default=256)
    ap.add_argument("--s", type=int, default=20)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import numpy as np
    from medane_tchakorom_ufc_thesis_repository_amd.petsc import Context, DenseMat, Mat, Vec
    ctx = Context(0)
    A = Mat.box_stencil_ext(ctx, 3, a.n, a.n, a.planes, True, True)
    nr, nc = A.shape
    S = DenseMat(ctx, nc, a.s)
    rng = np.random.default_rng(20251121)
    for j in range(a.s):
        S.set_column(j, 0, Vec.from_array(ctx, rng.uniform(-1, 1, nc)))
    R = DenseMat(ctx, nr, a.s)
    A.mat_mult_dense(S, R)
    ctx.set_timing(True, 1)
    ctx.reset_kernel_stats()
    for _ in range(a.reps):
        A.mat_mult_dense(S, R)
    st = ctx.kernel_stats()["spmm"]
    ctx.set_timing(False)
    h = hashlib.sha256(R.get_values().tobytes()).hexdigest()[:16]
    print(json.dumps({"cols_per_launch": os.environ.get("MSPLIT_SPMM_COLS", "default"), "launches": st["launches"],
                      "ms_per_product": st["ms"] / a.reps, "storage": A.get_storage(), "R_sha256_16": h}))


if __name__ == "__main__":
    main()
