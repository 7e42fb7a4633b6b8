"""Writes tests/golden/non_stencil_aij.json: the CPU oracle's GMRES on the non-stencil AIJ operator of bench.py's
non_stencil_aij line -- utils.heterogeneous_poisson3d(256), the 7-point -div(kappa grad u) with a per-cell kappa,
which keeps CSR storage --, b = A*1, x0 = 0, GMRES(30), pc none, unpreconditioned norm, rtol 1e-4, max_it 300, in
the DBR reduction order (the device's default), so the GPU box checks the timed step against it without running the
oracle.  Run from the repo root:  python tests/golden/make_non_stencil.py
"""
import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.join(HERE, "..", "..")
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, ROOT)
import pyoracle as po  # noqa: E402
from medane_tchakorom_ufc_thesis_repository_amd.utils import heterogeneous_poisson3d  # noqa: E402

N_EDGE, RESTART, MAX_IT, RTOL = 256, 30, 300, 1e-4


def main():
    po.build()
    po.set_threads(min(8, os.cpu_count() or 1))   # element-wise loops only: DBR dots are order-fixed
    rp, col, val = heterogeneous_poisson3d(N_EDGE)
    N = N_EDGE ** 3
    A = po.Mat.from_arrays(N, N, rp, col, val)
    b = A.mult(np.ones(N))
    t0 = time.time()
    x, r = po.gmres(A, b, restart=RESTART, max_it=MAX_IT, rtol=RTOL, reduce_mode=po.REDUCE_DBR)
    out = {"config": f"utils.heterogeneous_poisson3d({N_EDGE}) (CSR storage), b = A*1, x0 = 0, GMRES({RESTART}), "
                     f"pc none, rtol {RTOL}, max_it {MAX_IT}",
           "generator": "tests/golden/make_non_stencil.py (oracle/oracle.c, DBR order)",
           "csr_sha256": hashlib.sha256(rp.tobytes() + col.tobytes() + val.tobytes()).hexdigest(),
           "nnz": int(rp[-1]),
           "dbr": {"its": int(r["its"]), "reason": int(r["reason"]), "hist_hex": [float(h).hex() for h in r["hist"]],
                   "x_sha256": hashlib.sha256(np.ascontiguousarray(x, np.float64).tobytes()).hexdigest(),
                   "seconds": round(time.time() - t0, 1)}}
    json.dump(out, open(os.path.join(HERE, "non_stencil_aij.json"), "w"), indent=1)
    print(out["dbr"]["its"], out["dbr"]["reason"], out["dbr"]["seconds"], float.fromhex(out["dbr"]["hist_hex"][-1]))


if __name__ == "__main__":
    main()
