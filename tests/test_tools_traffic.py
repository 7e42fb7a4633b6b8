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
