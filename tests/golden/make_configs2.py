"""Writes tests/golden/configs2_smsm.json: the CPU oracle's SMSM-global (SMSM-global.c:288-363) with
BASELINE configs[2]'s exact options -- 2 z-slab blocks, s 20, inner GMRES(30) max_it 20 rtol 1e-20,
outer LSQR max_it 70 rtol 1e-15 with the exact matrix norm and the default convergence test, -rtol 1e-4
(running_bulk_test_g5k:230, :247-248) -- in the DBR order the device runs by default, up to configs[2] itself,
512^3.  From 512^3 on the oracle runs lean (orc_smsm_problem.lean: the operators applied without storage and
R = A S formed inside the LSQR, bit for bit the assembled run -- tests/test_oracle.py): S (21.5 GB) is its only
large array, so the record fits the container's memory; it takes the 8-thread oracle about 20 minutes per outer
iteration (ORC_PROGRESS=1 prints each one).

Per cube the record holds the outer count, norm0, every outer-history entry (hex), the LSQR counts and
reasons, the inner iteration counts, the final residual and the SHA-256 of x.  tests/test_gpu_configs.py
runs the same problem on the GPU and requires all of it bit for bit.

Run from the repo root:  python tests/golden/make_configs2.py [cube ...]      (default: 64 128 256)
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

NB, S, RTOL = 2, 20, 1e-4
INNER = dict(restart=30, max_it=20, rtol=1e-20, abstol=1e-50)
OUTER = dict(max_it=70, rtol=1e-15, abstol=1e-100, exact_norm=1, conv_test=0)
OUT = os.path.join(HERE, "configs2_smsm.json")


def record(n):
    t0 = time.time()
    r = po.smsm_solve(3, n, n, n, NB, S, RTOL, dict(INNER, reduce_mode=po.REDUCE_DBR),
                      dict(OUTER, reduce_mode=po.REDUCE_DBR), max_outer=40, lean=n >= 512)
    x = np.ascontiguousarray(r["x"], np.float64)
    return {"outer_its": int(r["outer_its"]), "norm0_hex": float(r["norm0"]).hex(),
            "hist_hex": [float(h).hex() for h in r["hist"]], "lsqr_its": [int(v) for v in r["lsqr_its"]],
            "lsqr_reason": [int(v) for v in r["lsqr_reason"]],
            "inner_its": r["inner_its"].tolist(), "total_inner_its": int(r["total_inner_its"]),
            "final_norm_hex": float(r["final_norm"]).hex(), "error": int(r["error"]),
            "x_sha256": hashlib.sha256(x.tobytes()).hexdigest(), "seconds": round(time.time() - t0, 1),
            **({"lean": True} if n >= 512 else {})}


def main():
    cubes = [int(a) for a in sys.argv[1:]] or [64, 128, 256]
    po.build()
    po.set_threads(min(8, os.cpu_count() or 1))   # element-wise loops only; DBR sums are order-fixed
    out = json.load(open(OUT)) if os.path.exists(OUT) else {}
    out.update({"config": "configs[2] options: 3D 7-pt Poisson, SMSM-global, 2 blocks, s 20, inner GMRES(30) max_it "
                          "20 rtol 1e-20, outer LSQR max_it 70 rtol 1e-15 exact norm, default test, -rtol 1e-4",
                "nb": NB, "s": S, "rtol": RTOL, "inner": INNER, "outer": OUTER, "reduce": "DBR",
                "generator": "tests/golden/make_configs2.py (oracle/oracle.c orc_smsm_solve)"})
    cubes_out = out.setdefault("cubes", {})
    for n in cubes:
        cubes_out[str(n)] = record(n)
        json.dump(out, open(OUT, "w"), indent=1)
        rec = cubes_out[str(n)]
        print(n, rec["outer_its"], rec["lsqr_its"], [float.fromhex(h) for h in rec["hist_hex"]], rec["seconds"],
              flush=True)


if __name__ == "__main__":
    main()
