"""Eager enqueue vs HIP-graph replay of GMRES restart cycles on small systems.

  python tools/graph_bench.py [--sizes 16,32,64,128] [--its 300]

One JSON line: per size, microseconds per Arnoldi step with MSPLIT_GRAPHS=0
and =1 (same process, interleaved, best of --rounds), timing off."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="16,32,64,128")
    ap.add_argument("--its", type=int, default=300)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    import torch  # noqa: F401
    from medane_tchakorom_ufc_thesis_repository_amd.petsc import KSP, Context, Mat, Options, Vec
    ctx = Context(0)
    out = {}
    for n in [int(v) for v in a.sizes.split(",")]:
        A = Mat.box_stencil(ctx, 3, n, n, n)
        N = n ** 3
        ones, b, x = Vec(ctx, N), Vec(ctx, N), Vec(ctx, N)
        ones.set(1.0)
        A.mult(ones, b)
        ksp = KSP(ctx)
        ksp.set_operators(A)
        ksp.set_from_options(Options(f"-ksp_gmres_restart 30 -ksp_max_it {a.its} -ksp_rtol 1e-300 -pc_type none"))
        best = {"0": 1e9, "1": 1e9}
        for _ in range(a.rounds):
            for g in ("0", "1"):
                os.environ["MSPLIT_GRAPHS"] = g
                ksp.solve(b, x)                   # warm (captures the cycle when graphs are on)
                ctx.synchronize()
                t0 = time.perf_counter()
                ksp.solve(b, x)
                ctx.synchronize()
                dt = time.perf_counter() - t0
                best[g] = min(best[g], dt / ksp.get_iteration_number() * 1e6)
        out[f"{n}^3"] = {"eager_us_per_step": best["0"], "graph_us_per_step": best["1"],
                         "speedup": best["0"] / best["1"]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
