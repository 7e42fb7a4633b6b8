"""Writes tests/golden/smsm_block.json: the CPU oracle's SMSM-global (SMSM-global.c:288-363) on exactly the block
bench.py's N = 1 SMSM lines time -- one 512 x 512 x 256 z-slab block, configs[2]'s options (s 20, inner GMRES(30)
max_it 20 rtol 1e-20, outer LSQR max_it 70 rtol 1e-15 with the exact matrix norm and the default test;
running_bulk_test_g5k:230, :247-248) -- from x = 0:

  dbr  3 outer iterations in the DBR order: smsm_per_gpu's warm-up step and its two timed steps;
  seq  1 outer iteration in PETSc's sequential order: the timed step of smsm_seq_mode.

Each holds every outer LSQR residual (hex), LSQR count and reason, every inner count and the SHA-256 of x after
the last iteration; bench.py checks its timed runs against them (check_smsm_block).  The oracle runs lean
(orc_smsm_problem.lean: bit for bit the assembled run, tests/test_oracle.py), so S is its only large array.

Run from the repo root:  ORC_PROGRESS=1 python tests/golden/make_smsm_block.py [dbr] [seq]
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

PROBLEM = {"dim": 3, "nx": 512, "ny": 512, "nz": 256, "nb": 1, "s": 20, "rtol": 1e-30}
INNER = dict(restart=30, max_it=20, rtol=1e-20, abstol=1e-100)
OUTER = dict(max_it=70, rtol=1e-15, abstol=1e-100, exact_norm=1, conv_test=0)
ORDERS = {"dbr": (po.REDUCE_DBR, 3), "seq": (po.REDUCE_SEQ, 1)}
OUT = os.path.join(HERE, "smsm_block.json")


def record(order, problem=PROBLEM):
    mode, outer_its = ORDERS[order]
    P = problem
    t0 = time.time()
    r = po.smsm_solve(P["dim"], P["nx"], P["ny"], P["nz"], P["nb"], P["s"], P["rtol"], dict(INNER, reduce_mode=mode),
                      dict(OUTER, reduce_mode=mode), max_outer=outer_its, lean=True)
    x = np.ascontiguousarray(r["x"], np.float64)
    return {"reduce": "DBR" if mode == po.REDUCE_DBR else "SEQ (PETSc's order)", "outer_its": int(r["outer_its"]),
            "norm0_hex": float(r["norm0"]).hex(), "hist_hex": [float(h).hex() for h in r["hist"]],
            "lsqr_its": [int(v) for v in r["lsqr_its"]], "lsqr_reason": [int(v) for v in r["lsqr_reason"]],
            "inner_its": [[int(v) for v in row.ravel()] for row in r["inner_its"]],
            "x_sha256": hashlib.sha256(x.tobytes()).hexdigest(), "seconds": round(time.time() - t0, 1)}


def main():
    orders = sys.argv[1:] or ["dbr", "seq"]
    po.build()
    po.set_threads(int(os.environ.get("ORC_THREADS", min(8, os.cpu_count() or 1))))  # element-wise loops, DBR chunks
    out = json.load(open(OUT)) if os.path.exists(OUT) else {}
    out.update({"problem": PROBLEM, "inner": INNER, "outer": OUTER,
                "generator": "tests/golden/make_smsm_block.py (oracle/oracle.c orc_smsm_solve, lean)"})
    for o in orders:
        out[o] = record(o)
        json.dump(out, open(OUT, "w"), indent=1)
        print(o, out[o]["lsqr_its"], [float.fromhex(h) for h in out[o]["hist_hex"]], out[o]["seconds"], flush=True)


if __name__ == "__main__":
    main()
