"""Writes tests/golden/smsm_ranks.json: the CPU oracle's SMSM-global (SMSM-global.c:288-363) on a small
3D 7-pt Poisson box split into nb z-slab blocks, for nb = 2..8, with the bench's inner/outer options
(GMRES(30) max_it 20, LSQR max_it 70 with the exact matrix norm) and a fixed number of outer iterations.

bench.py runs the same problem across its N ranks after the timed loop (one block per rank, over the
same library communicator the timed steps used: RCCL on the driver's node) and compares, bit for bit,
every rank's outer history, LSQR counts, final residual and the SHA-256 of its block of x with this record.
That is the N > 1 line's "verified" key: the multi-rank exchange, ordered sums and LSQR all-gathers
reproduce the single-process oracle.

Run from the repo root:  python tests/golden/make_smsm_ranks.py
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import pyoracle as po  # noqa: E402

# the problem: nx x ny x (planes * nb), s columns, a fixed number of outer iterations (rtol unreachable)
PROBLEM = {"dim": 3, "nx": 16, "ny": 12, "planes_per_block": 3, "s": 4, "outer_its": 3, "rtol": 1e-30}
INNER = dict(restart=30, max_it=20, rtol=1e-20, abstol=1e-100)
OUTER = dict(max_it=70, rtol=1e-15, abstol=1e-100, exact_norm=1, conv_test=0)


def record(nb):
    P = PROBLEM
    nx, ny, nz = P["nx"], P["ny"], P["planes_per_block"] * nb
    r = po.smsm_solve(3, nx, ny, nz, nb, P["s"], P["rtol"], dict(INNER, reduce_mode=po.REDUCE_DBR),
                      dict(OUTER, reduce_mode=po.REDUCE_DBR), max_outer=P["outer_its"])
    rows = nx * ny * P["planes_per_block"]
    x = np.ascontiguousarray(r["x"], np.float64)
    return {"outer_its": int(r["outer_its"]), "norm0_hex": float(r["norm0"]).hex(),
            "hist_hex": [float(h).hex() for h in r["hist"]], "lsqr_its": [int(v) for v in r["lsqr_its"]],
            "final_norm_hex": float(r["final_norm"]).hex(),
            "x_block_sha256": [hashlib.sha256(x[b * rows:(b + 1) * rows].tobytes()).hexdigest() for b in range(nb)]}


def main():
    po.build()
    out = {"problem": PROBLEM, "inner": INNER, "outer": OUTER, "reduce": "DBR",
           "generator": "tests/golden/make_smsm_ranks.py (oracle/oracle.c orc_smsm_solve)",
           "worlds": {str(nb): record(nb) for nb in range(2, 9)}}
    json.dump(out, open(os.path.join(HERE, "smsm_ranks.json"), "w"), indent=1)
    for nb, rec in out["worlds"].items():
        print(nb, rec["outer_its"], [float.fromhex(h) for h in rec["hist_hex"]])


if __name__ == "__main__":
    main()
