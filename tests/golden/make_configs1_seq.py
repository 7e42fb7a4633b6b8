"""Writes tests/golden/configs1_seq.json: the CPU oracle's GMRES on BASELINE configs[1] at full size
(3D 7-pt Poisson 256^3, b = A*1, x0 = 0, GMRES(30), pc none, 300 iterations) in PETSc's sequential
reduction order (ORC_REDUCE_SEQ), so the GPU box can check the device's MSP_REDUCE_SEQ mode against it
without running the ~2-minute single-threaded oracle.  Also records the same run in the DBR order and the
per-entry relative deviation between the two orders (the device's default mode is bitwise the DBR run,
tests/test_gpu_configs.py).

Run from the repo root:  python tests/golden/make_configs1_seq.py
"""
import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import pyoracle as po  # noqa: E402


def main():
    po.build()
    n, its = 256, 300
    po.set_threads(min(8, os.cpu_count() or 1))   # element-wise loops only: SEQ/DBR dots are order-fixed
    A = po.poisson3d_rows(n, n, n, 0, n)
    b = A.mult(np.ones(A.shape[0]))
    out = {"config": "configs[1]: 3D 7-pt Poisson 256^3, b = A*1, x0 = 0, GMRES(30), pc none, rtol 1e-30, "
                     "max_it 300", "generator": "tests/golden/make_configs1_seq.py (oracle/oracle.c)"}
    runs = {}
    for name, mode in (("seq", po.REDUCE_SEQ), ("dbr", po.REDUCE_DBR)):
        t0 = time.time()
        x, r = po.gmres(A, b, restart=30, max_it=its, rtol=1e-30, reduce_mode=mode)
        runs[name] = (x, r)
        out[name] = {"its": int(r["its"]), "reason": int(r["reason"]), "hist_hex": [float(h).hex() for h in r["hist"]],
                     "x_sha256": hashlib.sha256(np.ascontiguousarray(x, np.float64).tobytes()).hexdigest(),
                     "seconds": round(time.time() - t0, 1)}
    hs, hd = runs["seq"][1]["hist"], runs["dbr"][1]["hist"]
    rel = np.abs(hd - hs) / np.abs(hs)
    out["dbr_vs_seq"] = {"max_rel_dev_hist": float(rel.max()), "median_rel_dev_hist": float(np.median(rel)),
                         "max_abs_dev_over_r0": float((np.abs(hd - hs) / hs[0]).max()),
                         "max_rel_dev_x": float(np.max(np.abs(runs["dbr"][0] - runs["seq"][0]) /
                                                       np.abs(runs["seq"][0])))}
    json.dump(out, open(os.path.join(HERE, "configs1_seq.json"), "w"), indent=1)
    print(json.dumps(out["dbr_vs_seq"]), out["seq"]["seconds"], out["dbr"]["seconds"])


if __name__ == "__main__":
    main()
