"""tools/pmc_traffic.py's algorithmic bytes for the W-free GMRES step, on synthetic counter files (no GPU).

The PMC table under profiles/ compares each kernel class's HBM bytes with its algorithmic bytes; this pins the
accounting the tool applies to a GMRES(30) solve in dispatch order: the W-free MAXPY moves n + 8n(nv + 1)
(presence byte, x once, nv - 1 basis vectors, wout) at Arnoldi step nv, BuildSoln 8n(30 + 2), and the fused
MatMult+MDot without its W store 9n + 8n(nv - 1).
"""
import csv
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _write(d, counter, names):
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "run_counter_collection.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, ["Process_Id", "Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for i, nm in enumerate(names):
            w.writerow({"Process_Id": 1, "Dispatch_Id": i, "Kernel_Name": nm, "Counter_Name": counter,
                        "Counter_Value": 1.0})


@pytest.mark.parametrize("maxpy", ["k_box_maxpy_march", "k_box_maxpy"])
def test_wfree_accounting(tmp_path, maxpy):
    """Both W-free MAXPY kernels (marched tiles, and one chunk per workgroup where the fused kernel does not march)
    land in the maxpy class with the same algorithmic bytes."""
    n = 16
    N = float(n) ** 3
    names = []
    for _cycle in range(2):
        for it in range(30):
            names.append("void msk::k_box_spmv_mdot_march<1, true>(...)")
            names.append(f"void msk::{maxpy}<1, true>(...)")
        names.append("void msk::k_maxpy_chunk<true, false, 37>(...)")
    _write(str(tmp_path / "f"), "FETCH_SIZE", names)
    _write(str(tmp_path / "w"), "WRITE_SIZE", names)
    out = str(tmp_path / "traffic.json")
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_traffic.py"), str(tmp_path / "f"),
                    str(tmp_path / "w"), "--n", str(n), "--out", out], check=True, stdout=subprocess.DEVNULL)
    t = json.load(open(out))["classes"]
    maxpy = (sum(N + 8.0 * N * (nv + 1) for nv in range(1, 31)) + 8.0 * N * 32) / 31
    spmvdot = sum(9.0 * N + 8.0 * N * (nv - 1) for nv in range(1, 31)) / 30
    assert t["maxpy"]["launches"] == 62 and abs(t["maxpy"]["alg_bytes_per_launch"] / maxpy - 1) < 1e-12
    assert t["spmvdot"]["launches"] == 60 and abs(t["spmvdot"]["alg_bytes_per_launch"] / spmvdot - 1) < 1e-12


def test_smsm_per_kernel_accounting(tmp_path):
    """--smsm: the SMSM-global outer iteration's kernels on synthetic counters -- the W-free MAXPY and fused
    MatMult+MDot at Arnoldi steps 1..k of each of the s inner solves, BuildSoln, the LSQR GEMV (8n(s+2)) and
    x = S alpha (8n(s+1)) told apart by the template's AXPY argument, and the scaled dots (8n(s+1); the solve's
    first writes U = b / beta, 8n(s+2))."""
    nx, ny, nz, s, k = 8, 8, 4, 3, 5
    N = float(nx * ny * nz)
    names = []
    for _solve in range(s):
        for it in range(k):
            names.append("void msk::k_box_spmv_mdot_march<1, true>(...)")
            names.append("void msk::k_box_maxpy_march<1, true>(...)")
        names.append("void msk::k_maxpy_chunk<true, false, 37>(...)")
    names.append("void k_scaled_dot<true, 2, 4, true>(...)")       # the LSQR start: U = b / beta written
    for _step in range(4):
        names.append("void k_dense_gemv<true, true, 2, 4, true>(...)")
        names.append("void k_scaled_dot<true, 2, 4, true>(...)")
    names.append("void k_dense_gemv<false, false, 2, 4, true>(...)")
    _write(str(tmp_path / "f"), "FETCH_SIZE", names)
    _write(str(tmp_path / "w"), "WRITE_SIZE", names)
    out = str(tmp_path / "smsm.json")
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_traffic.py"), str(tmp_path / "f"),
                    str(tmp_path / "w"), "--smsm", f"{nx},{ny},{nz},{s},{k},4", "--out", out], check=True,
                   stdout=subprocess.DEVNULL)
    t = json.load(open(out))["kernels"]
    close = lambda a, b: abs(a / b - 1) < 1e-12  # noqa: E731
    assert t["k_box_maxpy_march"]["launches"] == s * k
    assert close(t["k_box_maxpy_march"]["alg_bytes_per_launch"], sum(N + 8 * N * (nv + 1) for nv in range(1, k + 1)) / k)
    assert close(t["k_box_spmv_mdot_march"]["alg_bytes_per_launch"], sum(9 * N + 8 * N * (nv - 1) for nv in range(1, k + 1)) / k)
    assert close(t["k_maxpy_chunk"]["alg_bytes_per_launch"], 8 * N * (k + 2))
    assert close(t["k_dense_gemv"]["alg_bytes_per_launch"], (4 * 8 * N * (s + 2) + 8 * N * (s + 1)) / 5)
    assert close(t["k_scaled_dot"]["alg_bytes_per_launch"], (8 * N * (s + 2) + 4 * 8 * N * (s + 1)) / 5)
