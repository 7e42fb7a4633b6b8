"""Writes tests/golden/smsm_seq.json: the CPU oracle's SMSM-global outer iteration on ONE z-slab block -- the
per-GPU workload of bench.py's N > 1 lines (configs[2]'s options: s 20, inner GMRES(30) max_it 20 rtol 1e-20,
outer LSQR max_it 70 rtol 1e-15 with the exact matrix norm and the default test; SMSM-global.c:288-363,
running_bulk_test_g5k:230, :247-248) -- in PETSc's sequential reduction order (ORC_REDUCE_SEQ), on a box small
enough for the single-threaded order: bench.py's smsm seq_mode line runs the same problem in the device's
MSP_REDUCE_SEQ mode and requires these bits (outer LSQR residual, LSQR count, inner counts, SHA-256 of x) before
it times the full-size block in that mode.

Run from the repo root:  python tests/golden/make_smsm_seq.py
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

PROBLEM = {"dim": 3, "nx": 48, "ny": 48, "nz": 32, "nb": 1, "s": 20, "outer_its": 1, "rtol": 1e-30}
INNER = dict(restart=30, max_it=20, rtol=1e-20, abstol=1e-100)
OUTER = dict(max_it=70, rtol=1e-15, abstol=1e-100, exact_norm=1, conv_test=0)


def record():
    """The record, computed now (tests/test_oracle.py checks the committed file against it)."""
    po.build()
    P = PROBLEM
    t0 = time.time()
    r = po.smsm_solve(P["dim"], P["nx"], P["ny"], P["nz"], P["nb"], P["s"], P["rtol"],
                      dict(INNER, reduce_mode=po.REDUCE_SEQ), dict(OUTER, reduce_mode=po.REDUCE_SEQ),
                      max_outer=P["outer_its"])
    x = np.ascontiguousarray(r["x"], np.float64)
    out = {"problem": PROBLEM, "inner": INNER, "outer": OUTER, "reduce": "SEQ (PETSc's order)",
           "generator": "tests/golden/make_smsm_seq.py (oracle/oracle.c orc_smsm_solve, ORC_REDUCE_SEQ)",
           "outer_its": int(r["outer_its"]), "norm0_hex": float(r["norm0"]).hex(),
           "hist_hex": [float(h).hex() for h in r["hist"]], "lsqr_its": [int(v) for v in r["lsqr_its"]],
           "inner_its": r["inner_its"].tolist(), "x_sha256": hashlib.sha256(x.tobytes()).hexdigest(),
           "seconds": round(time.time() - t0, 1)}
    return out


def main():
    out = record()
    json.dump(out, open(os.path.join(HERE, "smsm_seq.json"), "w"), indent=1)
    print(out["outer_its"], out["lsqr_its"], [float.fromhex(h) for h in out["hist_hex"]], out["seconds"])


if __name__ == "__main__":
    main()
