"""Where the exact parallel SEQ engine overtakes the serial one (MSP_REDUCE_SEQ).

Times a norm, a dot, an MDot over 30 vectors and one LSQR solve over 4 row blocks (the chained sums) at a range
of lengths, once per engine (MSPLIT_SEQ_ENGINE is read at every call).  Each line: one JSON object.
Run on the GPU box:  python tools/seq_crossover.py > gpurun_out/seq_crossover.jsonl
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from medane_tchakorom_ufc_thesis_repository_amd.petsc import LSQR, Context, DenseMat, Vec  # noqa: E402


def _time(fn, reps):
    fn()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    return (time.perf_counter() - t0) / reps


def main():
    c = Context(0)
    c.set_reduction("seq")
    rng = np.random.default_rng(5)
    for n in (1024, 4096, 8192, 16384, 32768, 65536, 131072, 262144, 524288, 1048576):
        x, y = Vec.from_array(c, rng.uniform(-1, 1, n)), Vec.from_array(c, rng.uniform(-1, 1, n))
        V = [Vec.from_array(c, rng.uniform(-1, 1, n)) for _ in range(30)]
        Rs = [rng.standard_normal((n // 4, 8)) for _ in range(4)]
        Rd = [DenseMat.from_array(c, R) for R in Rs]
        bs = [Vec.from_array(c, rng.standard_normal(n // 4)) for _ in range(4)]

        def lsqr():
            lq = LSQR(c)
            lq._set(max_it=10, rtol=1e-30, abstol=1e-300, exact_norm=1, conv_test=1)
            lq.set_operators(Rd)
            lq.solve(bs, Vec(c, 8))
            lq.destroy()

        reps = 20 if n <= 65536 else 4
        row = {"n": n}
        for eng in ("parallel", "serial"):
            os.environ["MSPLIT_SEQ_ENGINE"] = eng
            row[eng] = {"norm_us": 1e6 * _time(lambda: x.norm(), reps),
                        "dot_us": 1e6 * _time(lambda: x.dot(y), reps),
                        "mdot30_us": 1e6 * _time(lambda: x.mdot(V), reps),
                        "lsqr10_ms": 1e3 * _time(lsqr, max(1, reps // 4))}
        os.environ.pop("MSPLIT_SEQ_ENGINE")
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
