"""HBM traffic per launch from rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE).

  python tools/pmc_traffic.py FETCH_DIR WRITE_DIR --n 256 --out profiles/traffic.json

Correction applied as MI355X_MICROARCH.md section HBM prescribes for gfx950:
FETCH_SIZE (KiB) reports half the bytes of a wide coalesced streaming read,
so read bytes = 2 * FETCH_SIZE * 1024; WRITE_SIZE (KiB) is exact for 16-byte
stores.  Launches are grouped into the kernel classes bench.py reports; the
algorithmic bytes of each launch are recomputed from the kernel's template
arguments (the vector count) so the two can be compared launch for launch.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict


def wfree_maxpy(name: str) -> bool:
    """The W-free CGS MAXPY: k_box_maxpy_march (marched tiles) and k_box_maxpy (one chunk per workgroup: 2D boxes,
    planes without whole chunks, a ragged last chunk) -- the same bytes per launch."""
    return "k_box_maxpy" in name


def classify(name: str):
    if "spmv_mdot" in name:     # the GMRES MatMult fused with VecMDot (k_box_spmv_mdot[_march], k_spmv_mdot)
        return "spmvdot"
    if "k_maxpy" in name or wfree_maxpy(name):  # k_maxpy_chunk; the W-free CGS MAXPY k_box_maxpy[_march]
        return "maxpy"
    if "k_dot_stage1" in name:
        return "norm" if "true>" in name.replace(" ", "") or ", true" in name else "mdot"
    if "k_dot_stage2" in name:
        return "stage2"
    if "k_spmv" in name:
        return "spmv"
    if "k_blas1" in name:
        return "blas1"
    return "other"


def nv_of(name: str):
    m = re.search(r"k_(?:maxpy|dot_stage1)<(\d+)", name.replace(" ", ""))
    return int(m.group(1)) if m else None


def spmv_alg(name: str, n: int):
    """Algorithmic bytes of one SpMV launch on the n^3 7-point operator, by kernel and mode:
    DV-ELL W codes per row, CSR 12 per entry + rowptr; x read once, y written, b read in MatResidual."""
    nm = name.replace(" ", "")
    N = float(n) ** 3
    nnz = 7.0 * N - 6.0 * n * n
    m = re.search(r"k_spmv_ell<(\d+),(\d+),", nm)
    if m:
        mode, w = int(m.group(1)), int(m.group(2))
        return w * N + 16.0 * N + (8.0 * N if mode == 1 else 0.0)
    m = re.search(r"k_spmv_box_(?:march|lines)<(\d+),", nm)
    if m:  # the box-stencil march: one presence byte per row
        mode = int(m.group(1))
        return 1.0 * N + 16.0 * N + (8.0 * N if mode == 1 else 0.0)
    m = re.search(r"k_spmv_lds8<(\d+),", nm)
    if m:
        mode = int(m.group(1))
        return 12.0 * nnz + 4.0 * (N + 1) + 16.0 * N + (8.0 * N if mode == 1 else 0.0)
    return None


def base_name(name: str) -> str:
    """The kernel's function name: 'void msk::k_dense_gemv<true, ...>(...)' -> 'k_dense_gemv'."""
    nm = name.replace("(anonymous namespace)", "").split("(")[0].split("<")[0].split("::")[-1].split()
    return nm[-1] if nm else name


def tmpl_args(name: str):
    m = re.search(r"<([^<>]*)>", name)
    return [a.strip() for a in m.group(1).split(",")] if m else []


def smsm_alg(name: str, i: int, rows: float, s: int, k: int, lsqr: int = 70, onepass: bool = False):
    """Algorithmic bytes of the i-th launch (dispatch order) of this kernel in the SMSM-global per-GPU outer
    iteration (bench.py --variant smsm, SMSM-global.c:288-363): s inner GMRES solves of exactly k Arnoldi steps
    (rtol 1e-20) in the W-free step, then R = A S, the LSQR over R (n x s) of `lsqr` steps and x = S alpha, on
    `rows` rows."""
    N = rows
    b = base_name(name)
    if b == "k_box_maxpy_march" or b == "k_box_maxpy":
        return N + 8.0 * N * ((i % k) + 2)              # presence byte, x once, nv - 1 basis vectors, wout
    if b == "k_box_spmv_mdot_march" or b == "k_box_spmv_mdot":
        return 9.0 * N + 8.0 * N * (i % k)               # presence byte, x, nv - 1 basis vectors (W not stored)
    if b == "k_maxpy_chunk":
        return 8.0 * N * (k + 2)                         # BuildSoln: x += sum of k basis vectors
    if b == "k_dense_gemv":
        ax = tmpl_args(name)[:1] == ["true"]
        return 8.0 * N * (s + 2) if ax else 8.0 * N * (s + 1)   # U1 = R V - a U, ||U1||^2 / x = S alpha
    if b == "k_lsqr_onepass":  # the DBR LSQR step: R read once, U read, U1 written (its norm and R^T U1 from registers)
        return 8.0 * N * (s + 2)
    if b == "k_scaled_dot":   # R^T (U1 / beta), U1 not written back; the solve's first: U = b / beta written
        # (the one-pass step launches it only as each solve's first)
        return 8.0 * N * (s + 2) if onepass or i % (lsqr + 1) == 0 else 8.0 * N * (s + 1)
    return None


def smsm_table(fetch, write, rows, s, k, lsqr=70):
    """Per kernel: launches, HBM read/write bytes per launch (PMC) and the algorithmic bytes per launch."""
    per_f, per_w = defaultdict(list), defaultdict(list)
    for _, (name, v) in sorted(fetch.items()):
        per_f[base_name(name)].append((name, v))
    for _, (name, v) in sorted(write.items()):
        per_w[base_name(name)].append((name, v))
    out = {}
    for b in sorted(set(per_f) | set(per_w)):
        F, W = per_f.get(b, []), per_w.get(b, [])
        m = min(len(F), len(W))
        if m == 0:
            continue
        rd = sum(2.0 * v for _, v in F[:m]) / m
        wr = sum(v for _, v in W[:m]) / m
        als = [smsm_alg(nm, i, rows, s, k, lsqr, "k_lsqr_onepass" in per_f) for i, (nm, _) in enumerate(F[:m])]
        alg = sum(als) / m if all(a is not None for a in als) else None
        out[b] = {"launches": m, "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr,
                  "hbm_bytes_per_launch": rd + wr, "alg_bytes_per_launch": alg,
                  "hbm_over_alg": (rd + wr) / alg if alg else None}
    return out


def load(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    vals = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            key = (r.get("Process_Id", ""), int(r["Dispatch_Id"]))
            vals[key] = (r["Kernel_Name"], float(r["Counter_Value"]) * 1024.0)
    return vals


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--out", default="profiles/traffic.json")
    ap.add_argument("--bench", default=None, help="bench JSON of the same build: algorithmic bytes per launch")
    ap.add_argument("--x-reread", action="store_true",
                    help="builds before round 3's register dot: the fused kernel streamed x again for its dot")
    ap.add_argument("--smsm", default=None, metavar="NX,NY,NZ,S,K[,L]",
                    help="per-kernel table for the SMSM-global per-GPU outer iteration (bench.py --variant smsm): "
                         "an NX x NY x NZ block, S inner solves of K Arnoldi steps, L LSQR steps (70) over S columns")
    ap.add_argument("--kernel", default=None, metavar="NAME,ROW_BYTES",
                    help="one kernel of the GMRES(30) step only: every launch whose name contains NAME, in dispatch "
                         "order, against N x (ROW_BYTES + 8 x (i mod 30)) algorithmic bytes -- launch i of a cycle "
                         "dots W with i + 1 basis vectors, the last one from the march registers (e.g. "
                         "k_box_spmv_mdot_march_sym2,49: presence byte, 32 value bytes, x, W written)")
    a = ap.parse_args()
    N = a.n ** 3
    fetch = load(a.fetch_dir, "FETCH_SIZE")
    write = load(a.write_dir, "WRITE_SIZE")
    if a.kernel:
        name, row = a.kernel.split(",")
        F = [v for _, (nm, v) in sorted(fetch.items()) if name in nm]
        W = [v for _, (nm, v) in sorted(write.items()) if name in nm]
        m = min(len(F), len(W))
        hbm = [2.0 * F[i] + W[i] for i in range(m)]
        alg = [N * (float(row) + 8.0 * (i % 30)) for i in range(m)]
        out = {"kernel": name, "launches": m, "n": a.n, "row_bytes": float(row),
               "correction": "read = 2 x FETCH_SIZE x 1024 (gfx950), write = WRITE_SIZE x 1024",
               "hbm_bytes_per_launch": sum(hbm) / max(m, 1), "alg_bytes_per_launch": sum(alg) / max(m, 1),
               "hbm_over_alg": sum(hbm) / sum(alg) if m else None,
               "excess_bytes_per_launch": (sum(hbm) - sum(alg)) / max(m, 1)}
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        json.dump(out, open(a.out, "w"), indent=1)
        print(json.dumps(out, indent=1))
        return
    if a.smsm:
        f = [int(v) for v in a.smsm.split(",")]
        nx, ny, nz, s_, k_ = f[:5]
        l_ = f[5] if len(f) > 5 else 70
        out = {"workload": f"SMSM-global block {nx}x{ny}x{nz}, s {s_}, inner max_it {k_}, LSQR {l_} steps",
               "correction": "read = 2 x FETCH_SIZE x 1024 (gfx950), write = WRITE_SIZE x 1024",
               "kernels": smsm_table(fetch, write, float(nx) * ny * nz, s_, k_, l_)}
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        json.dump(out, open(a.out, "w"), indent=1)
        print(json.dumps(out, indent=1))
        return
    # dispatch ids of two runs of the same deterministic command line up per class and order
    per_class_f, per_class_w = defaultdict(list), defaultdict(list)
    for _, (name, v) in sorted(fetch.items()):
        per_class_f[classify(name)].append((name, v))
    for _, (name, v) in sorted(write.items()):
        per_class_w[classify(name)].append((name, v))
    out = {"n": a.n, "correction": "read = 2 x FETCH_SIZE x 1024 (gfx950), write = WRITE_SIZE x 1024",
           "classes": {}}
    for cls in sorted(set(per_class_f) | set(per_class_w)):
        F, W = per_class_f.get(cls, []), per_class_w.get(cls, [])
        m = min(len(F), len(W))
        if m == 0:
            continue
        rd = sum(2.0 * v for _, v in F[:m]) / m
        wr = sum(v for _, v in W[:m]) / m
        alg = None
        wfree = any(wfree_maxpy(nm) for nm, _ in F[:m]) or any(wfree_maxpy(nm) for nm, _ in
                                                                per_class_f.get("maxpy", []))
        if cls == "maxpy" and wfree and m % 31 == 0:
            # GMRES(30) solves in dispatch order: 30 W-free MAXPYs (presence byte, x once, nv - 1 basis vectors,
            # wout: N + 8 N (nv + 1), nv = it + 1), then BuildSoln's accumulate over 30 vectors (8 N (30 + 2))
            alg = sum(8.0 * N * 32 if not wfree_maxpy(nm) else N + 8.0 * N * ((i % 31) + 2)
                      for i, (nm, _) in enumerate(F[:m])) / m
        elif cls in ("maxpy", "mdot"):
            nvs = [nv_of(nm) for nm, _ in F[:m]]
            if all(nvs):
                k = 2 if cls == "maxpy" else 1
                alg = sum(8.0 * N * (nv + k) for nv in nvs) / m
        elif cls == "norm":
            alg = 8.0 * N
        elif cls == "spmvdot" and m % 30 == 0:
            # one GMRES(30) solve in dispatch order: the Arnoldi step it dots W with nv = it + 1 basis vectors; the
            # march's bytes (presence byte, x, W written) plus those vectors, W not re-read and the last vector
            # (x itself) dotted from the march's registers (round 3; --x-reread for builds before it)
            # (W-free builds: W is not written either, the MAXPY recomputes it)
            xr = 1 if a.x_reread else 0
            alg = sum((9.0 if wfree else 17.0) * N + 8.0 * N * ((i % 30) + xr) for i in range(m)) / m
        elif cls == "spmv":
            als = [spmv_alg(nm, a.n) for nm, _ in F[:m]]
            if all(als):
                alg = sum(als) / m
        out["classes"][cls] = {"launches": m, "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr,
                               "hbm_bytes_per_launch": rd + wr, "alg_bytes_per_launch": alg,
                               "hbm_over_alg": (rd + wr) / alg if alg else None}
    dom = "maxpy"
    if a.bench and os.path.exists(a.bench):
        b = json.load(open(a.bench))
        alg = b.get("roofline", {}).get("bytes_per_launch")
        if alg and dom in out["classes"]:
            out["classes"][dom]["alg_bytes_per_launch"] = alg
            out["classes"][dom]["hbm_over_alg"] = out["classes"][dom]["hbm_bytes_per_launch"] / alg
    if dom in out["classes"]:
        out["kernel_class"] = dom
        out["hbm_bytes_per_launch"] = out["classes"][dom]["hbm_bytes_per_launch"]
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
