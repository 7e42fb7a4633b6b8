"""Write profiles/r01/README.md and profiles/r01/final/* from a tools/gpu_round.sh run directory.

  python tools/profile_summary.py gpurun_out/<run> [--tag r01]
"""
from __future__ import annotations

import argparse
import csv
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("run")
    ap.add_argument("--tag", default="r01")
    ap.add_argument("--sub", default="final", help="directory under profiles/<tag>/ (its README.md is written there "
                                                   "unless --sub is final, which writes profiles/<tag>/README.md)")
    a = ap.parse_args()
    run = a.run
    D = os.path.join(ROOT, "profiles", a.tag, a.sub)
    os.makedirs(D, exist_ok=True)
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_traffic.py"), os.path.join(run, "pmc_fetch"),
                    os.path.join(run, "pmc_write"), "--n", "256", "--out", os.path.join(D, "traffic.json")],
                   check=True, stdout=subprocess.DEVNULL)
    shutil.copy(os.path.join(D, "traffic.json"), os.path.join(ROOT, "profiles", "traffic.json"))
    shutil.copy(os.path.join(run, "bench.json"), os.path.join(D, "bench.json"))
    shutil.copy(os.path.join(run, "bench_trace.json"), os.path.join(D, "bench_under_rocprof.json"))
    shutil.copy(os.path.join(run, "trace", "run_kernel_stats.csv"), os.path.join(D, "rocprofv3_kernel_stats.csv"))
    rows = list(csv.DictReader(open(os.path.join(D, "rocprofv3_kernel_stats.csv"))))
    b = json.loads(open(os.path.join(D, "bench.json")).read().strip().splitlines()[-1])
    bt = json.loads(open(os.path.join(D, "bench_under_rocprof.json")).read().strip().splitlines()[-1])
    tr = json.load(open(os.path.join(D, "traffic.json")))
    # the MAXPY class: the W-free k_box_maxpy_march (Arnoldi steps) and k_maxpy_chunk (BuildSoln); the class
    # average over both is what bench.py's HIP events time
    mxs = [r for r in rows if r["Name"] in ("k_box_maxpy_march", "k_maxpy_chunk")]
    calls = sum(int(r["Calls"]) for r in mxs)
    mx = {"Name": "+".join(r["Name"] for r in mxs), "Calls": calls,
          "AverageNs": sum(float(r["TotalDurationNs"]) for r in mxs) / calls}
    rf = b["roofline"]
    L = [f"# Round {a.tag[1:]} profiles (MI355X, gfx950, ROCm 7.2)", "",
         f"Command: `bash tools/gpu_round.sh {os.path.basename(run)}` (or tools/gpu_r02.sh, which adds smoke) = pytest -m gpu; `python bench.py`; "
         "`rocprofv3 --kernel-trace --stats -T -- python3 bench.py --steps 3 --no-cpu-baseline`;",
         "two PMC passes (`--pmc FETCH_SIZE`, `--pmc WRITE_SIZE`) of `bench.py --steps 1 --warmup 0 --no-timing`, "
         "reduced by `tools/pmc_traffic.py` (read = 2 x FETCH_SIZE on gfx950, write = WRITE_SIZE). "
         "Summary written by `tools/profile_summary.py`.", "",
         f"bench.py (N=1, 256^3, GMRES(30), 300 iterations/step): **{b['value']:.4g} DOF-updates/s**, "
         f"{b['ms_per_step']:.1f} ms/step; under rocprof: {bt['value']:.4g}.",
         f"cpu_baseline (oracle, {b['cpu_baseline']['cores']} host thread(s)): {b['cpu_baseline']['value']:.3g} DOF-updates/s"
         + (f"; single core {b['cpu_baseline']['single_core']['value']:.3g}" if 'single_core' in b['cpu_baseline'] else "")
         + ".", "",
         "## rocprofv3 --stats (4 solves = 1 warmup + 3 timed)", "",
         "| kernel | calls | total ms | avg us | % |", "|---|---|---|---|---|"]
    for r in rows:
        L.append(f"| {r['Name']} | {r['Calls']} | {int(r['TotalDurationNs']) / 1e6:.2f} | "
                 f"{float(r['AverageNs']) / 1e3:.2f} | {float(r['Percentage']):.2f} |")
    L += ["", "## Dominant kernel: bench.py's HIP-event timing vs rocprof", "",
          f"bench.py roofline (HIP events on {rf.get('timed_launches', 'every launch')}): class `maxpy` "
          f"({rf['kernel']}), avg {rf['avg_launch_ms'] * 1e3:.1f} us/launch, "
          f"{rf['bytes_per_launch'] / 1e9:.4f} GB algorithmic/launch -> {rf['achieved']:.0f} GB/s = "
          f"{rf['frac']:.3f} of 8 TB/s.",
          f"rocprof {mx['Name']}: avg {float(mx['AverageNs']) / 1e3:.1f} us over {mx['Calls']} calls "
          "(the class: the CGS MAXPY of each Arnoldi step and the BuildSoln accumulate launches).", "",
          "## HBM traffic per launch (PMC) vs algorithmic bytes", "",
          "| class | launches | HBM GB/launch | algorithmic GB/launch | ratio |", "|---|---|---|---|---|"]
    for k, v in tr["classes"].items():
        alg = v["alg_bytes_per_launch"]
        ratio = v["hbm_over_alg"]
        L.append(f"| {k} | {v['launches']} | {v['hbm_bytes_per_launch'] / 1e9:.4f} | "
                 f"{(alg / 1e9) if alg else float('nan'):.4f} | {ratio if ratio else float('nan'):.4f} |")
    L += ["", f"maxpy: n + 8n(k+1) (W-free) / 8n(k+2) (BuildSoln) algorithmic = {rf['bytes_per_launch'] / 1e9:.4f} GB/launch on average "
          f"(bench.py's figure), PMC {tr['hbm_bytes_per_launch'] / 1e9:.4f}.",
          (f"SpMV ({b['config'].get('matrix_storage', 'csr')} storage; GMRES's scaled form reads T once and writes "
           f"VV(it+1)): algorithmic {tr['classes']['spmv']['alg_bytes_per_launch'] / 1e9:.4f} GB/launch, PMC "
           f"{tr['classes']['spmv']['hbm_over_alg']:.2f}x (x rows read more than once: the z-march reads x(z+1) and the y-+1 lines, which miss L2 at the edges of an XCD run)."
           if tr['classes'].get('spmv', {}).get('alg_bytes_per_launch') else ""), "",
          "Other directories: `smsm/` (SMSM-global), `convdiff/`, `async/` (transports and async drivers), "
          "`configs/` (BASELINE configurations end to end), `spmv_ab/`, `skew_ab/`, `dv/`, `opfuse/`, `graphs/`, "
          "`matfree/`, A/Bs not adopted (`maxpy_pipe/`, `store_ab/`, `chunk_order/`, `dv/tried/`), earlier `*.json|csv` "
          "(first correct path, tuning history in DESIGN.md)."]
    mb = []
    for st in ("csr", "dv"):
        f = os.path.join(run, f"spmv512_{st}.json")
        if os.path.exists(f):
            shutil.copy(f, os.path.join(D, f"spmv512_{st}.json"))
            d = json.load(open(f))["spmv/t0/g0"]
            mb.append(f"| {st} | {d['us_median']:.1f} | {d['GBps_median']:.0f} | {d['GBps_median'] / 8000:.3f} |")
    if mb:
        L += ["", "## MatMult on the 512^3 7-point matrix (tools/microbench.py, y = A x, median of 3 x 10)", "",
              "| storage | us | algorithmic GB/s | of 8 TB/s |", "|---|---|---|---|"] + mb
    readme = os.path.join(ROOT, "profiles", a.tag, "README.md") if a.sub == "final" else os.path.join(D, "README.md")
    open(readme, "w").write("\n".join(L) + "\n")


if __name__ == "__main__":
    main()
