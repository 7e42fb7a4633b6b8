"""Writes tests/golden/*.json: the reference's own known-answer values
(src/tests/utils_test.c:76-228, copied as data) plus oracle vectors for the
GPU parity tests that must run without /root/reference.

Run from the repo root:  python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import pyoracle as po  # noqa: E402

kats = {
    "source": "reference src/tests/utils_test.c (data values only)",
    "residual_norm_golden": 2.54567588,
    "residual_inputs": {"x": {"0": [0.1234, 0.5678, 0.9101, 0.1121], "1": [0.8765, 0.4321, 0.5432, 0.6789]},
                        "b": {"0": [0.3141, 0.5926], "1": [0.2468, 0.1357]}},
    "poisson2d_2x2": {"0": [[4, -1, -1, 0], [-1, 4, 0, -1]], "1": [[-1, 0, 4, -1], [0, -1, -1, 4]]},
    "poisson3d_2x2x2": {"0": [[6, -1, -1, 0, -1, 0, 0, 0], [-1, 6, 0, -1, 0, -1, 0, 0],
                              [-1, 0, 6, -1, 0, 0, -1, 0], [0, -1, -1, 6, 0, 0, 0, -1]],
                        "1": [[-1, 0, 0, 0, 6, -1, -1, 0], [0, -1, 0, 0, -1, 6, 0, -1],
                              [0, 0, -1, 0, -1, 0, 6, -1], [0, 0, 0, -1, 0, -1, -1, 6]]},
}
json.dump(kats, open(os.path.join(HERE, "reference_kats.json"), "w"), indent=1)

# oracle GMRES histories (DBR and SEQ order) for a config-2-shaped small case
A = po.poisson3d_rows(16, 16, 16, 0, 16)
b = A.mult(np.ones(A.shape[0]))
out = {"problem": "3D 7-pt Poisson 16^3, b = A*1, x0 = 0, GMRES(30), pc none, rtol 1e-4, max_it 300"}
for name, mode in (("dbr", po.REDUCE_DBR), ("seq", po.REDUCE_SEQ)):
    x, r = po.gmres(A, b, restart=30, max_it=300, rtol=1e-4, reduce_mode=mode)
    out[name] = {"its": r["its"], "reason": r["reason"], "hist": [float.hex(float(h)) for h in r["hist"]],
                 "x_sum": float.hex(float(np.sum(x)))}
json.dump(out, open(os.path.join(HERE, "gmres_16cube.json"), "w"), indent=1)
print("golden fixtures written")
