"""Benchmark: DOF-updates/s of the GMRES inner solve on the 3D 7-point Poisson
operator (BASELINE.json metric), one process per GPU.

N = 1 : configs[1] -- 3D 7-pt Poisson 256^3, single-block GMRES(30), pc none,
        one step = one KSPSolve from x0 = 0 with the canonical options
        (running_bulk_test_g5k:64-70: rtol 1e-4, unpreconditioned norm) and a
        fixed max_it = 300 (10 restart cycles).
        The same JSON line also carries, each measured in this run:
          smsm_per_gpu  the N > 1 workload below on one GPU (one 512x512x256
                        block), so that N -> 8 compares SMSM with SMSM;
          spmv_512_csr  the north star's "CSR SpMV on the 512^3 7-point
                        matrix": MatMult with the matrix in CSR storage
                        (k_spmv_lds8), HIP-event time per launch and fraction
                        of the 8 TB/s HBM peak.
N > 1 : SMSM with global minimization (configs[2], BASELINE "SMSM 2 blocks on
        2 MI355X"), weak scaling: one 512 x 512 x 256 z-slab block per GPU
        (global 512 x 512 x 256N; N = 2 is the 512^3 two-block case).  One
        step = one outer iteration of SMSM-global.c:288-363 with the campaign
        options of running_bulk_test_g5k:230-248: s = 20 inner solves
        (GMRES(30), max_it 20, rtol 1e-20, warm started, boundary-plane
        exchange after each), S(:,k) = x, R = A S, LSQR (max_it 70,
        rtol 1e-15, exact Frobenius norm) and x = S alpha.  Exchange, residual
        sums and LSQR partials go over ONE library RCCL communicator on the
        context's stream (comm.LibComm; comm.c:126-141's replacement).
--variant sm    plain synchronous multisplitting (one z-slab block per GPU);
--variant amam  AMAM-global (asynchronous-multisplitting-asynchronous-
        minimization-global_prime.c:371-481): configs[3]'s per-GPU block of
        1024^3/8 = 1024x1024x128 (Poisson); with --peclet, configs[4]'s
        512^3/8 = 512x512x64 block of the convection-diffusion operator.  One
        step = one asynchronous solve of --amam-its outer iterations per block
        (HBM mailboxes, newest-value R broadcast, convergence detection).
value = sum over blocks of (rows x inner GMRES iterations) / max-over-ranks time.

Launch: python bench.py [--gpus N --steps K --warmup W]   (N > 1 under
torch.distributed.run, one rank per GPU, RCCL = backend "nccl").
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "DOF-updates/s on 3D 7-pt Poisson GMRES; achieved HBM GB/s vs peak, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0     # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
KERNEL_NAMES = {"mdot": "k_dot_stage1+2 (VecMDot, DBR)",
                "maxpy": "k_box_maxpy_march (VecMAXPY, CGS update with W = A(sc x) recomputed on the z-march + "
                         "fused ||w||^2) and k_maxpy_chunk (BuildSoln)",
                "norm": "k_dot_stage1<1,self>+stage2 (VecNorm)",
                "scale": "k_blas1<SCALE> (VecScale)", "other": "copy/set/axpy",
                "spmm": "k_spmm (MatMatMult R = A S)", "dgemv": "k_lsqr_onepass (LSQR step: R v - alpha u, its norm and R^T u in one pass over R; "
                                 "DBR default) / k_dense_gemv (S alpha; the two-pass step)",
                "dgemvt": "k_scaled_dot (LSQR's first R^T u; the two-pass step's scale + R^T u)",
                "spmvdot": "k_box_spmv_mdot_march (GMRES MatMult of the box stencil fused with VecMDot stage 1: "
                           "W not stored)"}
SPMV_NAMES = {"dv": "k_spmv_ell (MatMult/MatResidual, DV storage: one byte per entry)",
              "csr": "k_spmv_lds8 (MatMult/MatResidual, CSR storage)",
              "matfree": "k_stencil_spmv (MatMult/MatResidual, matrix-free)"}
MARCH_NAME = "k_spmv_box_march (MatMult/MatResidual, DV storage: one byte per entry; box stencil marched in z)"
LINES_NAME = ("k_spmv_box_lines (MatMult/MatResidual, DV storage: one byte per entry; box stencil marched in z "
              "over tiles of four y lines)")
CHUNK_NAME = ("k_box_march_chunk (MatMult/MatResidual, DV storage: one byte per entry; box stencil marched in z "
              "over DBR chunk tiles)")
TUNE_ELL_MARCH_OFF = 268435456


def spmv_name(storage, nx, ny=None):
    """The kernel the library picks for a box stencil's products (msk_spmv_box_march): the chunk-tile march
    where a plane holds whole 4096-row chunks, else the line or 256-row march."""
    tune = int(os.environ.get("MSPLIT_TUNING", "0") or 0)
    ny = nx if ny is None else ny
    if storage == "dv" and not tune & TUNE_ELL_MARCH_OFF:
        lines = os.environ.get("MSPLIT_MARCH_LINES", "0")
        fits = (nx * ny) % 4096 == 0 and nx % 2 == 0 and 2 <= nx <= 2048
        if fits and (lines == "16" or (lines == "0" and os.environ.get("MSPLIT_MARCH_CHUNK", "1") != "0")):
            return CHUNK_NAME
        return LINES_NAME if nx % 256 == 0 and lines != "1" else MARCH_NAME
    return SPMV_NAMES[storage]


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--mesh", type=int, default=256, help="mesh edge per block (256 -> configs[1])")
    p.add_argument("--max-it", type=int, default=300)
    p.add_argument("--restart", type=int, default=30)
    p.add_argument("--rtol", type=float, default=1e-4)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-sample-its", type=int, default=30)
    p.add_argument("--no-timing", action="store_true", help="disable per-kernel HIP-event timing")
    p.add_argument("--timing-every", type=int, default=7,
                   help="bracket one launch in N of each kernel class with HIP events (N = 1: every launch, "
                        "which costs ~2%% of the step in event records; 7 is co-prime with the restart 30, so the "
                        "samples cycle through every Krylov dimension)")
    p.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                   help="N>1 process group: nccl (= RCCL, the product) or gloo (single-GPU rehearsal: the library "
                        "communicator then uses its host transport over gloo)")
    p.add_argument("--variant", default=None, choices=["gmres", "sm", "smsm", "amam"],
                   help="gmres (N=1 default), smsm (N>1 default), sm, amam")
    p.add_argument("--smsm-mesh", type=int, default=512, help="SMSM: nx = ny")
    p.add_argument("--smsm-planes", type=int, default=256, help="SMSM: z-planes per GPU block")
    p.add_argument("--s", type=int, default=20, help="SMSM / AMAM: inner solves per minimization (-s)")
    p.add_argument("--inner-max-it", type=int, default=20)
    p.add_argument("--outer-max-it", type=int, default=70)
    p.add_argument("--amam-mesh", type=int, default=None, help="AMAM: nx = ny (1024; 512 with --peclet)")
    p.add_argument("--amam-planes", type=int, default=None, help="AMAM: z-planes per GPU (128; 64 with --peclet)")
    p.add_argument("--amam-its", type=int, default=2, help="AMAM: outer iterations per block per step")
    p.add_argument("--minimization", default="lsqr", choices=["lsqr", "rtr"],
                   help="AMAM: the replicated-R LSQR (outer_solver_norm_equation, utils.c:1061-1078; default) or "
                        "the reference's normal equations (outer_solver, utils.c:972-996: each block publishes "
                        "[R^T R | R^T b], s(s+1) doubles, instead of its rows of R)")
    p.add_argument("--operator", default="csr", choices=["csr", "matfree"],
                   help="the assembled operator (the reference's MatMult, default) or the same operator applied "
                        "matrix-free (bitwise the same products, no matrix traffic; gmres, and A_ii for smsm)")
    p.add_argument("--storage", default="dv", choices=["dv", "csr"],
                   help="entry storage of the assembled operator in HBM: dv (one byte per entry, the library's "
                        "choice for any matrix that fits; default) or csr (rowptr/col/val); bitwise the same products")
    p.add_argument("--no-csr-compare", action="store_true",
                   help="skip the CSR-storage rerun that N=1 GMRES reports beside the DV figure")
    p.add_argument("--no-smsm-n1", action="store_true", help="N=1: skip the smsm_per_gpu measurement")
    p.add_argument("--smsm-n1-steps", type=int, default=2)
    p.add_argument("--no-spmv512", action="store_true", help="N=1: skip the 512^3 CSR MatMult measurement")
    p.add_argument("--spmv-reps", type=int, default=20)
    p.add_argument("--no-seq-mode", action="store_true",
                   help="N=1: skip the seq_mode measurement (one configs[1] step in PETSc's reduction order)")
    p.add_argument("--no-seq-smsm", action="store_true",
                   help="N=1: skip the SMSM-global block outer iteration in PETSc's reduction order (verified first "
                        "on tests/golden/smsm_seq.json's small block)")
    p.add_argument("--no-non-stencil", action="store_true",
                   help="N=1: skip the non_stencil_aij measurement (GMRES on a per-cell-coefficient AIJ in CSR "
                        "storage, default and fused MatMult+MDot steps)")
    p.add_argument("--no-assembled", action="store_true",
                   help="N=1: skip the assembled_csr_operator measurement (the GMRES step with the operator handed "
                        "over as host CSR arrays, msp_mat_create_csr)")
    p.add_argument("--no-verify-ranks", action="store_true",
                   help="N>1: skip the post-timing multi-rank check (SMSM-global on a small box, one block per "
                        "rank over the same communicator, bitwise against tests/golden/smsm_ranks.json)")
    p.add_argument("--require-rccl", action="store_true",
                   help="N>1: exit non-zero when the library communicator could not be created over RCCL and the "
                        "run would fall back to the host transport (for the driver's scaling runs)")
    p.add_argument("--peclet", default=None,
                   help="Px,Py,Pz: the upwind convection-diffusion operator (configs[4]) instead of Poisson")
    a = p.parse_args()
    os.environ["MSPLIT_MAT_STORAGE"] = a.storage  # read by the library at each matrix assembly
    a.peclet = tuple(float(v) for v in a.peclet.split(",")) if a.peclet else None
    if a.peclet is not None and len(a.peclet) != 3:
        raise SystemExit("--peclet takes three cell Peclet numbers Px,Py,Pz")
    if a.amam_mesh is None:
        a.amam_mesh = 512 if a.peclet else 1024
    if a.amam_planes is None:
        a.amam_planes = 64 if a.peclet else 128
    return a


# ------------------------------------------------------------------ CPU baseline
def host_topology():
    """What the host offers: nproc, lscpu sockets/cores, this job's CPU set and cgroup quota."""
    out = {"nproc": os.cpu_count()}
    try:
        out["affinity_cpus"] = len(os.sched_getaffinity(0))
    except AttributeError:
        pass
    try:
        import subprocess
        txt = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        kv = {k.strip(): v.strip() for k, v in (ln.split(":", 1) for ln in txt.splitlines() if ":" in ln)}
        sockets = int(kv.get("Socket(s)", "0") or 0)
        cps = int(kv.get("Core(s) per socket", "0") or 0)
        out.update({"model": kv.get("Model name"), "sockets": sockets, "cores_per_socket": cps,
                    "physical_cores": sockets * cps, "threads_per_core": int(kv.get("Thread(s) per core", "1") or 1)})
    except Exception:
        pass
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        out["cgroup_cpu_quota"] = None if q == "max" else float(q) / float(per)
    except Exception:
        pass
    return out


def cpu_threads(topo):
    """This job's CPU share: the cgroup quota (the box grants each GPU job a share of the
    node), else the CPU set, else OMP_NUM_THREADS -- MSPLIT_CPU_THREADS overrides."""
    if os.environ.get("MSPLIT_CPU_THREADS"):
        return max(1, int(os.environ["MSPLIT_CPU_THREADS"]))
    share = topo.get("cgroup_cpu_quota") or topo.get("affinity_cpus") or topo.get("nproc") or 1
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    if omp > 0:
        share = min(share, omp)
    return max(1, int(share))


def cpu_baseline(n: int, restart: int, its: int, rtol: float):
    """The CPU restatement (oracle/) on a bounded sample of the same workload:
    the same 256^3 operator, GMRES(restart), pc none, from x0 = 0.  It runs with
    one thread per CPU of this job's share of the host (PETSc's MPI order with
    one rank per thread: element-wise loops split, each dot as per-thread pieces
    added in thread order), plus, for reference, one core in PETSc's Seq order."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import pyoracle as po
    topo = host_topology()
    threads = cpu_threads(topo)
    A = po.poisson3d_rows(n, n, n, 0, n)
    b = A.mult(np.ones(A.shape[0]))
    out = {}
    for t in ([threads, 1] if threads > 1 else [1]):
        po.set_threads(t)
        k = its * (8 if t > 1 else 1)
        t0 = time.perf_counter()
        _, r = po.gmres(A, b, restart=restart, max_it=k, rtol=rtol,
                        reduce_mode=po.REDUCE_MT if t > 1 else po.REDUCE_SEQ)
        dt = time.perf_counter() - t0
        out[t] = (A.shape[0] * r["its"] / dt, r["its"], dt)
    po.set_threads(1)
    v, k, dt = out[threads]
    res = {"value": v, "unit": "DOF-updates/s", "cores": threads, "kind": "port",
           "mode": ("OpenMP, one thread per CPU of the job's share, PETSc MPI dot order (one rank per thread)"
                    if threads > 1 else "one core, PETSc Seq order"),
           "sample": f"3D 7-pt Poisson {n}^3, GMRES({restart}) pc none, {k} iterations from x0=0, oracle/oracle.c "
                     f"(no FMA), {threads} thread(s), {dt:.1f} s",
           "host": topo}
    pc = topo.get("physical_cores")
    if pc and pc > threads:
        res["node_note"] = (f"the node has {pc} physical cores; this job's share is {threads} CPUs (the GPU box "
                            f"grants each single-GPU job a share of the host), so the baseline uses those")
    if threads > 1:
        v1, k1, dt1 = out[1]
        res["single_core"] = {"value": v1, "iterations": k1, "seconds": dt1, "order": "PETSc Seq"}
    return res


def load_ceiling():
    """The measured streaming ceiling of this MI355X model for the step's access mixes (tools/stream_ceiling.hip:
    plain 16-byte non-temporal read / copy / MAXPY-mix kernels, profiles/r03/stream_ceiling/), or None."""
    p = os.path.join(ROOT, "profiles", "r03", "stream_ceiling", "n256.json")
    try:
        d = json.load(open(p))
    except Exception:
        return None
    return {"read_TBps": max(d["read8_TBps"], d["read16_TBps"]), "copy_TBps": d["copy_TBps"],
            "maxpy_mix_TBps": max(d["mix15_TBps"], d["mix15_u8_TBps"]),
            "source": "profiles/r03/stream_ceiling/n256.json (tools/stream_ceiling.hip, 256^3 vectors)"}


def load_traffic():
    """HBM bytes per launch of the dominant kernel from the committed PMC summary
    (tools/pmc_traffic.py over rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this
    benchmark), or None.  Read from profiles/, not counted in this run: rocprofv3's
    counter passes cannot run inside the timed process."""
    p = os.path.join(ROOT, "profiles", "traffic.json")
    if not os.path.exists(p):
        return None
    try:
        return json.load(open(p))
    except Exception:
        return None


# ------------------------------------------------------------------ workloads
def smsm_options(args):
    return (f"-inner1_ksp_type gmres -inner1_ksp_gmres_restart {args.restart} -inner1_ksp_atol 1e-100 "
            f"-inner1_ksp_max_it {args.inner_max_it} -inner1_ksp_rtol 1e-20 -inner1_pc_type none "
            f"-inner1_ksp_norm_type UNPRECONDITIONED "
            f"-outer1_ksp_type lsqr -outer1_ksp_convergence_test default -outer1_ksp_lsqr_exact_mat_norm "
            f"-outer1_ksp_atol 1e-100 -outer1_ksp_max_it {args.outer_max_it} -outer1_ksp_rtol 1e-15 "
            f"-outer1_pc_type none -outer1_ksp_norm_type UNPRECONDITIONED -s {args.s}"
            + (" -msplit_operator matfree" if args.operator == "matfree" else ""))


def build_smsm(ctx, args, comm, world, rank):
    """configs[2]: SMSM-global (SMSM-global.c:288-363), options of running_bulk_test_g5k:230-248."""
    from medane_tchakorom_ufc_thesis_repository_amd.multisplitting import GpuBlock, GpuMinimizer
    from medane_tchakorom_ufc_thesis_repository_amd.petsc import Options
    from medane_tchakorom_ufc_thesis_repository_amd.utils import block_layout
    n = args.smsm_mesh
    nz = args.smsm_planes * world
    kspopts = smsm_options(args)
    o = Options(kspopts)
    L = block_layout(3, n, n, nz, world, rank, args.peclet)
    blk = GpuBlock(ctx, L, o, comm, prefix="inner1_")
    blk.setup_minimization(args.s)
    mini = GpuMinimizer(ctx, [blk], comm, o, prefix="outer1_")
    blk.reset_halo()
    lsqr_its = []
    lsqr_rnorm = []                         # KSPGetResidualNorm of each step's LSQR: the outer history
    inner_its = []

    def step():
        its = 0
        for k in range(args.s):
            blk.update_rhs()                # updateLocalRHS
            k_its = blk.solve()             # inner_solver
            its += k_its
            inner_its.append(k_its)
            comm.exchange([blk])            # comm_sync_send_and_receive
            blk.store_column(k)             # S(:, k) = x
        blk.form_R()                        # R = A S
        rn, lits, _ = mini.solve([blk])     # LSQR, x = S alpha
        lsqr_its.append(lits)
        lsqr_rnorm.append(rn)
        return its
    transport = {"local": "single block", "nccl": "one library RCCL communicator",
                 "gloo": "gloo (rehearsal: the library's host transport)"}[getattr(comm, "backend", "local")]
    if getattr(comm, "backend", None) == "nccl" and getattr(comm, "transport", "rccl") != "rccl":
        transport = "the library's host transport over the NCCL process group (RCCL communicator unavailable)"
    workload = (f"3D 7-pt Poisson {n}x{n}x{nz} SMSM-global, {world} z-slab block(s) of {n}x{n}x{args.smsm_planes} "
                f"(one per MI355X), s = {args.s} inner GMRES({args.restart}) solves of max_it {args.inner_max_it} "
                f"per outer iteration, LSQR max_it {args.outer_max_it}; {transport} for the exchange, residual sums "
                f"and LSQR partials (configs[2] at N = 2)")
    step.lsqr_rnorm, step.inner_its, step.lsqr_its = lsqr_rnorm, inner_its, lsqr_its
    return step, workload, kspopts, n * n * args.smsm_planes, (blk, mini, lsqr_its)


SMSM_BLOCK_GOLDEN = os.path.join(ROOT, "tests", "golden", "smsm_block.json")


def smsm_block_record(args, order):
    """The committed oracle record of exactly the N = 1 SMSM block (tests/golden/smsm_block.json, written by
    tests/golden/make_smsm_block.py: one 512 x 512 x 256 z-slab block, configs[2]'s options, outer iterations from
    x = 0 in the DBR order -- the smsm_per_gpu warm-up and timed steps -- and one in PETSc's order -- the
    smsm_seq_mode step), or None when the bench runs another block."""
    if not os.path.exists(SMSM_BLOCK_GOLDEN):
        return None
    g = json.load(open(SMSM_BLOCK_GOLDEN))
    P, inn, out = g["problem"], g["inner"], g["outer"]
    if (args.smsm_mesh, args.smsm_planes, args.s, args.inner_max_it, args.outer_max_it, args.restart) != (
            P["nx"], P["nz"], P["s"], inn["max_it"], out["max_it"], inn["restart"]) or args.peclet is not None:
        return None
    return g.get(order)


C2_GOLDEN = os.path.join(ROOT, "tests", "golden", "configs2_smsm.json")


def check_configs2_run(args, step, rank):
    """(verified, mismatches, outer iterations checked): an N = 2 SMSM run is configs[2] (512^3, two z-slab blocks
    of 512 x 512 x 256, configs[2]'s options) -- its first outer iterations against the oracle record of that
    problem: LSQR residual (hex), LSQR count, and this rank's inner counts.  (None, ...) for another problem."""
    if not os.path.exists(C2_GOLDEN):
        return None, ["no record"], 0
    g = json.load(open(C2_GOLDEN))
    rec = g.get("cubes", {}).get("512")
    if (rec is None or (args.smsm_mesh, args.smsm_planes, args.s, args.inner_max_it, args.outer_max_it,
                        args.restart) != (512, 256, g["s"], g["inner"]["max_it"], g["outer"]["max_it"],
                                          g["inner"]["restart"]) or args.peclet is not None):
        return None, ["not configs[2]'s problem"], 0
    k = min(len(step.lsqr_rnorm), len(rec["hist_hex"]))
    bad = []
    if [float(h).hex() for h in step.lsqr_rnorm[:k]] != rec["hist_hex"][:k]:
        bad.append("hist_hex")
    if list(step.lsqr_its[:k]) != rec["lsqr_its"][:k]:
        bad.append("lsqr_its")
    if step.inner_its[:k * args.s] != [rec["inner_its"][o][j][rank] for o in range(k) for j in range(args.s)]:
        bad.append("inner_its")
    return not bad, bad, k


def check_smsm_block(step, blk, ref, nsteps):
    """(verified, mismatches): the first nsteps outer iterations of an SMSM block run against its oracle record --
    every LSQR residual (hex), LSQR count and inner count, and the SHA-256 of x after the last one."""
    import hashlib
    import numpy as np
    if ref is None:
        return None, ["no record for this block"]
    if nsteps > len(ref["hist_hex"]):
        return None, [f"record holds {len(ref['hist_hex'])} outer iterations, the run did {nsteps}"]
    bad = []
    if [float(h).hex() for h in step.lsqr_rnorm[:nsteps]] != ref["hist_hex"][:nsteps]:
        bad.append("hist_hex")
    if list(step.lsqr_its[:nsteps]) != ref["lsqr_its"][:nsteps]:
        bad.append("lsqr_its")
    want_inner = [v for outer in ref["inner_its"][:nsteps] for v in outer]
    if step.inner_its[:len(want_inner)] != want_inner:
        bad.append("inner_its")
    if nsteps == len(ref["hist_hex"]):
        xs = hashlib.sha256(np.ascontiguousarray(blk.x.get_array(), np.float64).tobytes()).hexdigest()
        if xs != ref["x_sha256"]:
            bad.append("x_sha256")
    return not bad, bad


def smsm_n1(ctx, args):
    """The N > 1 per-GPU workload on this one GPU (LocalComm, one block): the base the
    driver's N = 2..8 SMSM lines scale from."""
    import torch
    from medane_tchakorom_ufc_thesis_repository_amd.comm import LocalComm
    step, workload, _, rows, (blk, mini, lsqr_its) = build_smsm(ctx, args, LocalComm(), 1, 0)
    step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    its = sum(step() for _ in range(args.smsm_n1_steps))
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    # after timing: the warm-up and every timed outer iteration against the DBR oracle record of this block
    ok, bad = check_smsm_block(step, blk, smsm_block_record(args, "dbr"), 1 + args.smsm_n1_steps)
    mini.close()
    return {"workload": workload, "value": rows * its / dt, "unit": "DOF-updates/s", "steps": args.smsm_n1_steps,
            "warmup": 1, "ms_per_step": 1e3 * dt / args.smsm_n1_steps,
            "gmres_iterations_per_step": its / args.smsm_n1_steps, "lsqr_iterations_per_step": lsqr_its[1:],
            "verified": ok, "mismatch": bad,
            "reference": "tests/golden/smsm_block.json['dbr'] (oracle/oracle.c orc_smsm_solve, DBR order, lean): "
                         "every outer LSQR residual (hex), LSQR and inner count of the warm-up and timed steps, and "
                         "the SHA-256 of x after them",
            "note": "same per-GPU block and step as the N > 1 lines: N-GPU scaling of SMSM = "
                    "value(N) / (N x this value)"}


def spmv512(ctx, args):
    """The north star's SpMV target: MatMult y = A x on the 512^3 7-point matrix in CSR
    storage (rowptr/col/val; 12 B per entry), HIP events on the library's stream."""
    import numpy as np
    import torch
    from medane_tchakorom_ufc_thesis_repository_amd.petsc import Mat, Vec
    n = 512
    A = Mat.box_stencil(ctx, 3, n, n, n)
    A.set_storage("csr")
    N = A.shape[0]
    x = Vec.from_array(ctx, np.random.default_rng(20251121).uniform(-1, 1, N))
    y = Vec(ctx, N)
    for _ in range(3):
        A.mult(x, y)
    ctx.set_timing(True, 1)
    ctx.reset_kernel_stats()
    for _ in range(args.spmv_reps):
        A.mult(x, y)
    st = ctx.kernel_stats()["spmv"]
    ctx.set_timing(False)
    torch.cuda.synchronize()
    alg = 12.0 * A.nnz + 20.0 * N + 4.0
    avg_ms = st["ms"] / st["launches"]
    gbs = alg / (avg_ms * 1e-3) / 1e9
    A.destroy()
    # after timing: the last product against MatMult_SeqAIJ's row sums restated in numpy (bit for bit)
    xs, ys = x.get_array(), y.get_array()
    bad_rows = sum(int(np.count_nonzero(poisson3d_rows_product(xs, n, z).view(np.uint64)
                                        != ys[z * n * n:(z + 1) * n * n].view(np.uint64))) for z in range(n))
    return {"kernel": SPMV_NAMES["csr"], "rows": N, "nnz": A.nnz, "alg_bytes_per_launch": alg,
            "verified": bad_rows == 0, "mismatched_rows": bad_rows,
            "verification": "the last timed product, every row bit for bit against MatMult_SeqAIJ's ordered row sums "
                            "restated in numpy",
            "bytes_formula": "12 nnz + 20 N + 4 (val 8 + col 4 per entry, rowptr, x read once, y written)",
            "launches": st["launches"], "avg_launch_ms": avg_ms, "achieved_GBps": gbs,
            "peak_GBps": HBM_PEAK_GBS, "frac": gbs / HBM_PEAK_GBS, "target_frac": 0.70}


def poisson3d_rows_product(xs, n, z):
    """Plane z of y = A x for the n^3 7-point Poisson matrix (utils.c:30-121) as MatMult_SeqAIJ forms each row: from
    0.0, the row's entries in column order (z-1, y-1, x-1, d, x+1, y+1, z+1), one product and one add each, no FMA --
    numpy's element-wise double arithmetic, so bit for bit what the CSR kernel must give."""
    import numpy as np
    P = n * n
    o = z * P
    idx = np.arange(P)
    i, j = idx % n, idx // n
    acc = np.zeros(P)

    def add(mask, src):
        nonlocal acc
        t = np.zeros(P)
        t[mask] = (-1.0) * xs[src[mask]]
        acc = np.where(mask, acc + t, acc)
    if z > 0:
        acc = acc + (-1.0) * xs[o - P:o]
    add(j > 0, o + idx - n)
    add(i > 0, o + idx - 1)
    acc = acc + 6.0 * xs[o:o + P]
    add(i < n - 1, o + idx + 1)
    add(j < n - 1, o + idx + n)
    if z < n - 1:
        acc = acc + (-1.0) * xs[o + P:o + 2 * P]
    return acc


GOLDEN = os.path.join(ROOT, "tests", "golden", "configs1_seq.json")


def golden_configs1(args, n):
    """The committed oracle result of exactly this GMRES step (tests/golden/configs1_seq.json:
    configs[1], b = A*1, x0 = 0, GMRES(30), 300 iterations; "dbr" = the default reduction
    order, "seq" = PETSc's), or None when the bench runs another workload."""
    if not (n == 256 and args.max_it == 300 and args.restart == 30 and args.peclet is None
            and args.rtol <= 1e-4 and os.path.exists(GOLDEN)):
        return None
    return json.load(open(GOLDEN))


def verify_ranks(ctx, comm, world, rank):
    """The N > 1 line's check, after the timed loop: SMSM-global on the small box of
    tests/golden/smsm_ranks.json, one z-slab block per rank over the SAME library communicator the
    timed steps used (RCCL on the driver's node: grouped ncclSend/ncclRecv planes, ncclAllGather of the
    residual sums and LSQR partials), compared bit for bit with the single-process oracle's record for
    this world size (outer history, LSQR counts, final residual, SHA-256 of this rank's block of x).
    Returns (ok, mismatch list, seconds); every rank gets the all-ranks verdict."""
    import hashlib
    import numpy as np
    import torch.distributed as dist
    from medane_tchakorom_ufc_thesis_repository_amd.multisplitting import make_smsm, smsm_solve
    from medane_tchakorom_ufc_thesis_repository_amd.petsc import Options
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tests", "golden", "smsm_ranks.json")
    if not os.path.exists(path):
        return None, ["no record"], 0.0
    g = json.load(open(path))
    ref = g["worlds"].get(str(world))
    if ref is None:
        return None, [f"no record for {world} ranks"], 0.0
    P, inn, out = g["problem"], g["inner"], g["outer"]
    opts = " ".join(f"-inner{b + 1}_ksp_type gmres -inner{b + 1}_ksp_gmres_restart {inn['restart']} "
                    f"-inner{b + 1}_ksp_max_it {inn['max_it']} -inner{b + 1}_ksp_rtol {inn['rtol']} "
                    f"-inner{b + 1}_ksp_atol {inn['abstol']} -inner{b + 1}_pc_type none "
                    f"-outer{b + 1}_ksp_type lsqr -outer{b + 1}_ksp_convergence_test default "
                    f"-outer{b + 1}_ksp_lsqr_exact_mat_norm -outer{b + 1}_ksp_atol {out['abstol']} "
                    f"-outer{b + 1}_ksp_max_it {out['max_it']} -outer{b + 1}_ksp_rtol {out['rtol']} "
                    f"-outer{b + 1}_pc_type none" for b in range(world))
    t0 = time.perf_counter()
    nz = P["planes_per_block"] * world
    blocks, mini = make_smsm(ctx, 3, P["nx"], P["ny"], nz, world, [rank], P["s"], Options(f"{opts} -s {P['s']}"),
                             comm)
    res = smsm_solve(blocks, comm, P["s"], mini, rtol=P["rtol"], max_outer=P["outer_its"])
    xs = hashlib.sha256(np.ascontiguousarray(blocks[0].x.get_array(), np.float64).tobytes()).hexdigest()
    mini.close()
    got = {"outer_its": res.outer_its, "norm0_hex": float(res.norm0).hex(),
           "hist_hex": [float(h).hex() for h in res.hist], "lsqr_its": [int(v) for v in res.lsqr_its],
           "final_norm_hex": float(res.final_norm).hex()}
    bad = [k for k in got if got[k] != ref[k]]
    if xs != ref["x_block_sha256"][rank]:
        bad.append("x_block_sha256")
    allbad = [None] * world
    dist.all_gather_object(allbad, bad)
    mismatch = [f"rank {r}: {k}" for r, b in enumerate(allbad) for k in b]
    return not mismatch, mismatch, time.perf_counter() - t0


def check_step(ksp, x, ref):
    """Compare one GMRES step's result (iteration count, reason, every history entry as hex,
    SHA-256 of x) with a committed oracle record; outside any timed region."""
    import hashlib
    import numpy as np
    hist = [float(h).hex() for h in ksp.get_residual_history()]
    xs = hashlib.sha256(np.ascontiguousarray(x.get_array(), np.float64).tobytes()).hexdigest()
    got = {"its": ksp.get_iteration_number(), "reason": ksp.get_converged_reason(), "hist_hex": hist,
           "x_sha256": xs}
    bad = [k for k in ("its", "reason", "hist_hex", "x_sha256") if got[k] != ref[k]]
    return not bad, bad


def assembled_operator_step(ctx, args, b, ref):
    """The GMRES step with the operator handed over as host CSR arrays through msp_mat_create_csr -- the path
    the PETSc plugin's MatAssemblyEnd / KSPSetUp take for the reference's assembled AIJ (poisson3DMatrix,
    utils.c:30-121, cut by MatCreateSubMatrix, :450-478).  The arrays are the assembled 256^3 operator
    (downloaded from a device assembly: the same rows, columns and values); the library recognises the box
    stencil and attaches the z-march SpMV.  Timed over the same steps and checked against the oracle record."""
    import torch
    from medane_tchakorom_ufc_thesis_repository_amd.petsc import KSP, Mat, Options, Vec
    n = args.mesh
    A0 = Mat.box_stencil(ctx, 3, n, n, n)
    rp, col, val = A0.get_csr()
    A0.destroy()
    N = n * n * n
    t0 = time.perf_counter()
    A = Mat.from_csr(ctx, N, N, rp, col, val)
    create_s = time.perf_counter() - t0
    del rp, col, val
    ksp = KSP(ctx)
    ksp.set_operators(A)
    ksp.set_from_options(Options(f"-ksp_type gmres -ksp_gmres_restart {args.restart} -pc_type none "
                                 f"-ksp_norm_type unpreconditioned -ksp_rtol {args.rtol} -ksp_max_it {args.max_it}"))
    ksp.set_initial_guess_nonzero(False)
    x = Vec(ctx, N)
    ksp.solve(b, x)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    its = 0
    for _ in range(args.steps):
        ksp.solve(b, x)
        its += ksp.get_iteration_number()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t1
    ok = check_step(ksp, x, ref["dbr"])[0] if ref is not None else None
    out = {"operator": "host CSR arrays through msp_mat_create_csr (the PETSc plugin's path)",
           "spmv_kernel": A.spmv_kernel(), "matrix_storage": A.get_storage(), "value": float(N) * its / dt,
           "unit": "DOF-updates/s", "ms_per_step": 1e3 * dt / args.steps, "steps": args.steps,
           "create_s": create_s, "verified": ok}
    A.destroy()
    return out


NON_STENCIL_GOLDEN = os.path.join(ROOT, "tests", "golden", "non_stencil_aij.json")


def non_stencil_step(ctx, args):
    """The GMRES step on an assembled AIJ no dictionary covers: utils.heterogeneous_poisson3d(256), the 7-point
    -div(kappa grad u) with a per-cell kappa (every row holds its own values), as host CSR arrays through
    msp_mat_create_csr -- the general operator a PETSc user hands over; b = A*1, x0 = 0, GMRES(30), 300
    iterations.  Timed three ways on the same matrix: the storage the library picks (STENCIL: the box stencil's
    presence byte and each row's seven values, the chunk-tile march, the MatMult fused with the VecMDot with W
    stored), CSR storage (k_spmv_lds8, then the CGS kernels), and CSR with the MatMult fused with the VecMDot
    (k_spmv_mdot, MSK_TUNE_GM_SPMV_MDOT).  Each is checked against the committed oracle record
    (tests/golden/non_stencil_aij.json, written by tests/golden/make_non_stencil.py)."""
    import torch
    from medane_tchakorom_ufc_thesis_repository_amd import _lib
    from medane_tchakorom_ufc_thesis_repository_amd.petsc import KSP, Mat, Options, Vec
    from medane_tchakorom_ufc_thesis_repository_amd.utils import heterogeneous_poisson3d
    n = 256
    ref = json.load(open(NON_STENCIL_GOLDEN)) if os.path.exists(NON_STENCIL_GOLDEN) else None
    rp, col, val = heterogeneous_poisson3d(n)
    N = n ** 3
    t0 = time.perf_counter()
    A = Mat.from_csr(ctx, N, N, rp, col, val)
    create_s = time.perf_counter() - t0
    nnz = int(rp[-1])
    del rp, col, val
    ones = Vec(ctx, N)
    ones.set(1.0)
    b = Vec(ctx, N)
    A.mult(ones, b)
    ksp = KSP(ctx)
    ksp.set_operators(A)
    ksp.set_from_options(Options("-ksp_type gmres -ksp_gmres_restart 30 -pc_type none -ksp_norm_type "
                                 "unpreconditioned -ksp_rtol 1e-4 -ksp_max_it 300"))
    ksp.set_initial_guess_nonzero(False)
    x = Vec(ctx, N)
    L = _lib.load()
    L.msk_set_tuning.argtypes = [ctypes.c_int]
    L.msk_set_tuning.restype = None
    L.msk_get_tuning.restype = ctypes.c_int
    saved = int(L.msk_get_tuning())   # MSPLIT_TUNING as the context applied it: restored after every variant
    picked = A.get_storage()
    out = {"operator": "utils.heterogeneous_poisson3d(256): 7-point -div(kappa grad u), per-cell kappa, host CSR "
                       "through msp_mat_create_csr", "rows": N, "nnz": nnz, "matrix_storage": picked,
           "spmv_kernel": A.spmv_kernel(), "create_s": create_s,
           "reference": "tests/golden/non_stencil_aij.json['dbr']"}
    steps = max(1, min(args.steps, 3))
    variants = [("default", picked, saved), ("csr_storage", "csr", saved), ("csr_fused_matmult_mdot", "csr", saved | 2048)]
    for name, storage, flags in variants:
        A.set_storage(storage)
        L.msk_set_tuning(flags)
        try:
            ksp.solve(b, x)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            its = 0
            for _ in range(steps):
                ksp.solve(b, x)
                its += ksp.get_iteration_number()
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            ok, bad = check_step(ksp, x, ref["dbr"]) if ref else (None, ["no record"])
        finally:
            L.msk_set_tuning(saved)
        out[name] = {"matrix_storage": storage, "value": float(N) * its / dt, "unit": "DOF-updates/s",
                     "ms_per_step": 1e3 * dt / steps, "steps": steps, "verified": ok, "mismatch": bad}
    A.set_storage(picked)
    out["value"] = out["default"]["value"]
    out["verified"] = all(out[k]["verified"] for k, _, _ in variants)
    A.destroy()
    return out


def seq_mode_step(ctx, ksp, b, x, ref):
    """One configs[1] step with every reduction in PETSc's sequential order (MSP_REDUCE_SEQ, the parity
    mode -msplit_reduction seq selects), timed and checked against the PETSc-order oracle record."""
    import torch
    ctx.set_reduction("seq")
    try:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ksp.solve(b, x)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        its = ksp.get_iteration_number()
        ok, bad = check_step(ksp, x, ref["seq"]) if ref else (None, [])
    finally:
        ctx.set_reduction("dbr")
    return {"reduction": "seq (PETSc's order: one running sum per dot/norm/MDot entry)",
            "engine": ("serial (one lane adds in order)" if os.environ.get("MSPLIT_SEQ_ENGINE", "")[:1] in ("s", "S")
                       else "exact parallel (msplit_seq.hip: binade transducers of 64-term subs and 4096-term "
                            "segments, applied in order as ripples through a wave, the f64 add where the sum leaves "
                            "its binade; short sums take the serial engine: norms below 2^13 terms, dots 2^17, MDots 2^19)"),
            "value": float(x.n) * its / dt, "unit": "DOF-updates/s", "seconds_per_step": dt,
            "gmres_iterations": its, "verified": ok, "mismatch": bad,
            "reference": "tests/golden/configs1_seq.json['seq'] (oracle/oracle.c ORC_REDUCE_SEQ)",
            "note": "the parity mode: identical iteration counts and bitwise PETSc-order histories, at this cost "
                    "(47.97 s per step with the serial engine, round 3; 5.40 s with round 5's scan walk)"}


SMSM_SEQ_GOLDEN = os.path.join(ROOT, "tests", "golden", "smsm_seq.json")


def smsm_seq_mode(ctx, args):
    """The N > 1 per-GPU workload (one SMSM-global outer iteration on one z-slab block: s inner GMRES solves, R = A S,
    the LSQR, x = S alpha) with every reduction in PETSc's sequential order (-msplit_reduction seq).  First the same
    step on the small block of tests/golden/smsm_seq.json (written by the PETSc-order oracle), compared bit for bit;
    then one outer iteration of the full-size block, timed."""
    import hashlib
    import numpy as np
    import torch
    from medane_tchakorom_ufc_thesis_repository_amd.comm import LocalComm
    from medane_tchakorom_ufc_thesis_repository_amd.multisplitting import smsm_solve
    g = json.load(open(SMSM_SEQ_GOLDEN)) if os.path.exists(SMSM_SEQ_GOLDEN) else None
    out = {"reduction": "seq (PETSc's order)", "workload": None, "verified": None, "mismatch": []}
    ctx.set_reduction("seq")
    try:
        if g is not None:
            P = g["problem"]
            a2 = argparse.Namespace(**vars(args))
            a2.smsm_mesh, a2.smsm_planes, a2.s = P["nx"], P["nz"], P["s"]
            a2.inner_max_it, a2.outer_max_it = g["inner"]["max_it"], g["outer"]["max_it"]
            a2.restart, a2.peclet, a2.operator = g["inner"]["restart"], None, "csr"
            _, _, _, _, (blk, mini, _) = build_smsm(ctx, a2, LocalComm(), 1, 0)
            res = smsm_solve([blk], LocalComm(), P["s"], mini, rtol=P["rtol"], max_outer=P["outer_its"])
            got = {"outer_its": res.outer_its, "norm0_hex": float(res.norm0).hex(),
                   "hist_hex": [float(h).hex() for h in res.hist], "lsqr_its": [int(v) for v in res.lsqr_its],
                   "inner_its": np.array(res.inner_its).tolist(),
                   "x_sha256": hashlib.sha256(np.ascontiguousarray(blk.x.get_array(), np.float64).tobytes())
                   .hexdigest()}
            mini.close()
            del blk, mini
            out["mismatch"] = [k for k in got if got[k] != g[k]]
            out["verified"] = not out["mismatch"]
            out["reference"] = "tests/golden/smsm_seq.json (oracle/oracle.c orc_smsm_solve, ORC_REDUCE_SEQ)"
        step, workload, _, rows, (blk, mini, lsqr_its) = build_smsm(ctx, args, LocalComm(), 1, 0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        its = step()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        # after timing: the timed full-size outer iteration against the PETSc-order oracle record of this block
        ok_full, bad_full = check_smsm_block(step, blk, smsm_block_record(args, "seq"), 1)
        mini.close()
    finally:
        ctx.set_reduction("dbr")
    out["small_block"] = {"verified": out["verified"], "mismatch": out["mismatch"]}
    out["verified"] = (ok_full if out["verified"] is None else (out["verified"] and ok_full)
                       if ok_full is not None else None)
    out["mismatch"] = out["mismatch"] + [f"full block: {m}" for m in bad_full]
    out.update({"workload": workload, "value": rows * its / dt, "unit": "DOF-updates/s", "seconds_per_step": dt,
                "gmres_iterations": its, "lsqr_iterations": lsqr_its[-1],
                "full_block_reference": "tests/golden/smsm_block.json['seq'] (oracle/oracle.c orc_smsm_solve, "
                                        "ORC_REDUCE_SEQ, lean): the LSQR residual (hex), LSQR and inner counts and "
                                        "the SHA-256 of x of the timed outer iteration",
                "note": "the parity mode on the SMSM block (configs[2]'s per-GPU workload): one outer iteration"})
    return out


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("--gpus N > 1 needs torch.distributed.run with N processes")
    ndev = max(1, torch.cuda.device_count())
    dev = local_rank % ndev                  # identity on a full node; rehearsals may share a GPU
    torch.cuda.set_device(dev)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group("gloo")
    from medane_tchakorom_ufc_thesis_repository_amd.comm import LibComm, LocalComm
    from medane_tchakorom_ufc_thesis_repository_amd.multisplitting import GpuBlock
    from medane_tchakorom_ufc_thesis_repository_amd.petsc import KSP, Context, Mat, Options, Vec
    from medane_tchakorom_ufc_thesis_repository_amd.utils import block_layout

    n = args.mesh
    stream = torch.cuda.current_stream().cuda_stream
    ctx = Context(dev, stream=stream)
    kspopts = (f"-ksp_type gmres -ksp_gmres_restart {args.restart} -pc_type none -ksp_norm_type unpreconditioned "
               f"-ksp_rtol {args.rtol} -ksp_max_it {args.max_it}")
    rows = n * n * n
    variant = args.variant or ("gmres" if world == 1 else "smsm")
    if variant == "gmres" and world > 1:
        raise SystemExit("--variant gmres is the single-GPU workload")
    comm = LibComm(ctx) if world > 1 else LocalComm()
    transport = getattr(comm, "transport", "none") if world > 1 else "none"
    if args.require_rccl and world > 1 and transport != "rccl":
        # every rank agreed on the same transport (LibComm), so every rank exits here
        print(f"bench.py: --require-rccl, but the library communicator runs over the {transport} transport",
              file=sys.stderr, flush=True)
        comm.close()
        dist.destroy_process_group()
        sys.exit(3)
    keep = None
    spmv_storage = "matfree" if args.operator == "matfree" else args.storage

    if variant == "gmres":
        # configs[1]: single-block GMRES(30) on 256^3 (gmres_solution.c:50-70 in 3D)
        if args.operator == "matfree":
            A = Mat.box_matfree(ctx, 3, n, n, n, False, False, args.peclet)
        else:
            A = Mat.box_convdiff(ctx, 3, n, n, n, False, False, args.peclet or (0.0, 0.0, 0.0))
        ones = Vec(ctx, rows)
        ones.set(1.0)
        b = Vec(ctx, rows)
        A.mult(ones, b)
        x = Vec(ctx, rows)
        ksp = KSP(ctx)
        ksp.set_operators(A)
        ksp.set_from_options(Options(kspopts))
        ksp.set_initial_guess_nonzero(False)
        ksp.set_up()

        def step():
            ksp.solve(b, x)                     # zero initial guess: x is reset by KSPSolve
            return ksp.get_iteration_number()
        workload = f"3D 7-pt Poisson {n}^3, single-block GMRES({args.restart}) on 1 MI355X (configs[1])"
        if args.operator == "matfree":
            workload += ", operator applied matrix-free (same arithmetic as the CSR; not the reference's MatMult)"
    elif variant == "sm":
        L = block_layout(3, n, n, n * world, world, rank, args.peclet)
        o = Options(kspopts)
        blk = GpuBlock(ctx, L, None, comm, prefix="")
        blk.ksp.set_from_options(o)
        blk.reset_halo()
        blk.update_rhs()

        def step():
            its = blk.solve()                   # inner_solver (warm start, UIRNorm)
            comm.exchange([blk])
            blk.update_rhs()
            sq = blk.local_residual_sq()
            comm.ordered_sum([blk], [sq])
            return its
        workload = (f"3D 7-pt Poisson {n}x{n}x{n * world} synchronous multisplitting, {world} z-slab blocks of "
                    f"{n}^3 (one per MI355X), inner GMRES({args.restart}) max_it {args.max_it}, "
                    f"{'library RCCL communicator' if world > 1 else 'single block'}")
    elif variant == "amam":
        # configs[3] / configs[4]: AMAM-global, one block per GPU (AMAM-global_prime.c:371-481)
        from medane_tchakorom_ufc_thesis_repository_amd.asynchronous import am_solve
        n = args.amam_mesh
        nz = args.amam_planes * world
        kspopts = smsm_options(args)
        o = Options(kspopts)
        L = block_layout(3, n, n, nz, world, rank, args.peclet)
        blk = GpuBlock(ctx, L, o, comm, prefix="inner1_")
        blk.setup_global_async_minimization(args.s, o, prefix="outer1_", minimization=args.minimization)
        rows = L.nrows
        amres = []

        def step():
            r = am_solve([blk], comm, rtol=1e-30, max_iterations=args.amam_its, variant="amam_global", s=args.s,
                         stop_at_limit=True)
            amres.append(r)
            return sum(r.inner_its)
        workload = (f"3D 7-pt {'upwind convection-diffusion' if args.peclet else 'Poisson'} {n}x{n}x{nz} AMAM-global, "
                    f"{world} z-slab block(s) of {n}x{n}x{args.amam_planes} (one per MI355X; "
                    f"{'configs[4]' if args.peclet else 'configs[3]'} per-GPU block), s = {args.s} inner GMRES("
                    f"{args.restart}) steps of max_it {args.inner_max_it}, {args.amam_its} outer iterations per block "
                    f"per step, LSQR max_it {args.outer_max_it} "
                    + ("over the replicated R" if args.minimization == "lsqr" else
                       "on R^T R (outer_solver: Gram parts broadcast)") + ", HBM mailboxes (xGMI)")
        keep = amres
    else:
        step, workload, kspopts, rows, (blk, mini, lsqr_its) = build_smsm(ctx, args, comm, world, rank)
        n = args.smsm_mesh

    if args.peclet is not None:
        workload = workload.replace("7-pt Poisson", "7-pt upwind convection-diffusion (cell Peclet "
                                    + ",".join(f"{v:g}" for v in args.peclet) + ")")
        workload = workload.replace("(configs[1])", "(configs[1] shape, configs[4] operator)")

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    for _ in range(args.warmup):
        step()
    timing = not args.no_timing
    ctx.set_timing(timing, args.timing_every)
    ctx.reset_kernel_stats()
    barrier()
    t0 = time.perf_counter()
    its_total = 0
    for _ in range(args.steps):
        its_total += step()
    barrier()
    elapsed = time.perf_counter() - t0
    stats = ctx.kernel_stats() if timing else {}

    # the result of the last timed step against the committed oracle record (outside the timed region)
    verified, mismatch, ref_ranks = None, [], None
    ref = golden_configs1(args, n) if variant == "gmres" and world == 1 else None
    if ref is not None:
        verified, mismatch = check_step(ksp, x, ref["dbr"])

    csr_same_run = None
    if (variant == "gmres" and world == 1 and args.operator == "csr" and args.storage == "dv"
            and not args.no_csr_compare):
        # the same workload with the matrix in CSR storage, same process, same timing setting
        A.set_storage("csr")
        step()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        its_c = sum(step() for _ in range(args.steps))
        torch.cuda.synchronize()
        el_c = time.perf_counter() - t1
        A.set_storage("dv")
        ok_c = check_step(ksp, x, ref["dbr"])[0] if ref is not None else None
        csr_same_run = {"matrix_storage": "csr", "value": float(rows) * its_c / el_c,
                        "ms_per_step": 1e3 * el_c / args.steps, "verified": ok_c,
                        "timing": f"HIP events 1 in {args.timing_every}" if timing else "off"}
    ctx.set_timing(False)

    my_updates = float(rows) * its_total
    if world > 1:
        t = torch.tensor([elapsed, my_updates], dtype=torch.float64,
                         device="cuda" if args.backend == "nccl" else "cpu")
        tmax = t.clone()
        dist.all_reduce(tmax[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(t[1:], op=dist.ReduceOp.SUM)
        elapsed_max, updates = float(tmax[0]), float(t[1])
        timed_check = None
        if variant == "smsm" and world == 2:
            # N = 2 is configs[2] itself (512^3, two blocks): the run's own outer iterations -- warm-up and timed --
            # against the oracle record of that problem, as far as the record goes (it ends where configs[2]
            # converges); every rank checks its block's inner counts, the verdict is all ranks'
            ok_t, bad_t, nchk = check_configs2_run(args, step, rank)
            if ok_t is not None:
                flag = torch.tensor([0.0 if ok_t else 1.0], dtype=torch.float64,
                                    device="cuda" if args.backend == "nccl" else "cpu")
                dist.all_reduce(flag, op=dist.ReduceOp.SUM)
                ok_t = float(flag[0]) == 0.0
            timed_check = {"verified": ok_t, "mismatch": bad_t, "outer_iterations_checked": nchk,
                           "outer_iterations_run": args.warmup + args.steps,
                           "reference": "tests/golden/configs2_smsm.json['cubes']['512'] (oracle/oracle.c "
                                        "orc_smsm_solve, DBR order, lean): every outer LSQR residual (hex), LSQR "
                                        "count and inner count of the run's first outer iterations"}
        if not args.no_verify_ranks:
            # collective on every rank, after the timed loop and outside it
            verified, vmis, vsec = verify_ranks(ctx, comm, world, rank)
            ref_ranks = {"reference": "tests/golden/smsm_ranks.json (oracle/oracle.c orc_smsm_solve, DBR order)",
                         "checked": f"SMSM-global on a small box, {world} z-slab blocks, one per rank over this "
                                    f"run's library communicator ({transport}): outer history (hex), LSQR counts, "
                                    "final residual, SHA-256 of every rank's block of x",
                         "mismatch": vmis, "seconds": round(vsec, 3)}
    else:
        elapsed_max, updates = elapsed, my_updates

    extras = {}
    if world == 1 and variant == "gmres" and rank == 0:
        if not args.no_seq_mode and ref is not None:
            extras["seq_mode"] = seq_mode_step(ctx, ksp, b, x, ref)
        if not args.no_assembled and args.operator == "csr" and args.peclet is None:
            extras["assembled_csr_operator"] = assembled_operator_step(ctx, args, b, ref)
        if not args.no_non_stencil and args.operator == "csr" and args.peclet is None and n == 256:
            extras["non_stencil_aij"] = non_stencil_step(ctx, args)
        # release the headline's objects, then the two side measurements
        del ksp, A, b, x, ones
        if not args.no_spmv512:      # before the SMSM block's ~30 GB come and go
            extras["spmv_512_csr"] = spmv512(ctx, args)
        if not args.no_smsm_n1:
            extras["smsm_per_gpu"] = smsm_n1(ctx, args)
        if not args.no_seq_smsm:
            extras["smsm_seq_mode"] = smsm_seq_mode(ctx, args)

    if rank == 0:
        value = updates / elapsed_max
        mesh = {"gmres": [n, n, n], "sm": [n, n, n], "smsm": [n, n, args.smsm_planes],
                "amam": [args.amam_mesh, args.amam_mesh, args.amam_planes]}[variant]
        out = {"metric": METRIC, "value": value, "unit": "DOF-updates/s", "n_gpus": world, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": 1e3 * elapsed_max / args.steps, "higher_is_better": True,
               "scaling": "weak", "vs_baseline": None, "dtype": "f64",
               "data": "synthetic: b = A*1 (exact solution u = 1), x0 = 0; device-assembled operator",
               "config": {"workload": workload, "variant": variant, "mesh_per_gpu": mesh, "blocks": world,
                          "ksp": kspopts, "gmres_iterations_per_step_per_block": its_total / args.steps / world,
                          "matrix_storage": "none (matrix-free)" if args.operator == "matfree" else args.storage,
                          "parallelism": f"{world} z-slab block(s), one per GPU",
                          "transport": transport},
               "verified": verified}
        if ref_ranks is not None:
            out["verification"] = ref_ranks
        if world > 1 and timed_check is not None:
            out["timed_run_verification"] = timed_check
            if timed_check["verified"] is False:
                verified = False
                out["verified"] = False
        if ref is not None:
            out["verification"] = {"reference": "tests/golden/configs1_seq.json['dbr'] (oracle/oracle.c, DBR order)",
                                   "checked": "iterations, reason, every residual-history entry (hex), SHA-256 of x",
                                   "mismatch": mismatch}
        if variant == "smsm":
            out["config"]["lsqr_iterations_per_step"] = lsqr_its[-args.steps:]
        if variant == "amam":
            out["config"]["amam"] = [{"iterations": r.iterations, "inner_its": r.inner_its, "converged": r.converged,
                                      "transport": r.transport,
                                      "phase_share": {k: v / max(sum(r.timers.values()), 1e-30)
                                                      for k, v in r.timers.items()}} for r in keep[-args.steps:]]
        if csr_same_run:
            out["same_run_csr_storage"] = csr_same_run
        if stats:
            total_ms = sum(s["ms"] for s in stats.values())
            dom = max(stats, key=lambda k: stats[k]["ms"])
            s = stats[dom]
            achieved = (s["bytes"] / s["launches"]) / (s["ms"] / s["launches"] * 1e-3) / 1e9 if s["launches"] else 0
            tr = load_traffic()
            ceil = load_ceiling()
            traffic = None
            if tr and tr.get("kernel_class") == dom and tr.get("n") == n and variant == "gmres":
                traffic = tr.get("hbm_bytes_per_launch")
            names = dict(KERNEL_NAMES, spmv=spmv_name(spmv_storage, n))
            out["roofline"] = {"bound": "hbm", "kernel": names[dom], "achieved": achieved,
                               "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                               "traffic": traffic,
                               "traffic_source": ("profiles/traffic.json: rocprofv3 --pmc FETCH_SIZE/WRITE_SIZE "
                                                  "passes of this benchmark (tools/pmc_traffic.py, gfx950 "
                                                  "correction), read from profiles/, not counted in this run"
                                                  if traffic is not None else None),
                               "timed_launches": f"1 in {args.timing_every} per class",
                               "measured_ceiling": ceil,
                               "frac_of_measured_read_ceiling": (achieved / (1e3 * ceil["read_TBps"])
                                                                 if ceil else None),
                               "bytes_per_launch": s["bytes"] / max(s["launches"], 1),
                               "avg_launch_ms": s["ms"] / max(s["launches"], 1)}
            out["kernels"] = {k: {"kernel": names.get(k, k), "launches": v["launches"], "ms_total": v["ms"],
                                  "GBps": (v["bytes"] / (v["ms"] * 1e-3) / 1e9) if v["ms"] else None,
                                  "share": v["ms"] / total_ms if total_ms else None} for k, v in stats.items()}
            alg_bytes = sum(v["bytes"] for v in stats.values())
            # sampled launches stand for timing_every launches each
            out["hbm_alg_GBps_whole_step"] = alg_bytes * max(1, args.timing_every) / elapsed / 1e9
        out.update(extras)
        if world == 1 and variant == "gmres" and not args.no_cpu_baseline and args.peclet is None:
            out["cpu_baseline"] = cpu_baseline(n, args.restart, args.cpu_sample_its, args.rtol)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    failed = (verified is False or (extras.get("seq_mode") or {}).get("verified") is False
              or (extras.get("smsm_per_gpu") or {}).get("verified") is False
              or (extras.get("spmv_512_csr") or {}).get("verified") is False
              or (extras.get("smsm_seq_mode") or {}).get("verified") is False
              or (extras.get("assembled_csr_operator") or {}).get("verified") is False
              or (extras.get("non_stencil_aij") or {}).get("verified") is False)
    if variant == "smsm":
        mini.close()
    if world > 1:
        comm.close()                            # the library communicator before the process group
        dist.barrier()
        dist.destroy_process_group()
    if failed:
        print("bench.py: the timed step's result differs from the committed oracle record", file=sys.stderr)
        sys.exit(1)


if __name__ == "__main__":
    main()
