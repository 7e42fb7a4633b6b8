"""nb = 8: the world size of BASELINE configs[3], configs[4] and the driver's 8-GPU scaling bench.

The reference hard-wires 2 blocks (iSolve:332-338, utils.c:42-54, conv_detection.c:180-196); the build
generalises the split, the exchange, the ordered sums, the LSQR partials and the detection to nb blocks.
These tests run that generalisation at nb = 8 in every form the one-GPU box allows:

* SM and SMSM-global with 8 blocks in one process (LocalComm), bitwise the DBR oracle -- and SMSM-global on
  tests/golden/smsm_ranks.json's problem bitwise its committed 8-block record (the record bench.py checks
  its N = 8 ranks against after timing);
* the C host with one block per MPI rank at 8 ranks, over the host transport and over RCCL (one NCCL_HOSTID
  per rank: RCCL's socket transport on this one GPU), bitwise the same record, every rank's block of x
  included;
* AMAM-global round-robin at nb = 8 (Poisson and convection-diffusion, both minimizations), bitwise the twin
  (oracle/am_twin.py);
* the whole of configs[4]: all 8 blocks of the 512^3 convection-diffusion AMAM-global run round-robin on the
  one GPU (rtr), to termination, with a bitwise rerun.
"""
import gc
import hashlib
import json
import os
import tempfile

import numpy as np
import pytest

import am_twin
from medane_tchakorom_ufc_thesis_repository_amd.asynchronous import am_solve
from medane_tchakorom_ufc_thesis_repository_amd.comm import LocalComm
from medane_tchakorom_ufc_thesis_repository_amd.multisplitting import make_blocks, make_smsm, sm_solve, smsm_solve
from medane_tchakorom_ufc_thesis_repository_amd.petsc import ConvDetection, Options

from test_gpu_c_drivers import SM, SMSM, _run, _run_rccl, built  # noqa: F401  (built: the C host fixture)

# eight ranks on the one GPU, one hardware queue each: with HIP's four, eight ranks and this GPU-using pytest parent
# oversubscribe the GPU's 24 compute-queue slots and the scheduler runs them a process at a time
# (tests/test_gpu_async_mp.py, profiles/r06/async8/)
ONE_QUEUE = {"GPU_MAX_HW_QUEUES": "1"}

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
RANKS = json.load(open(os.path.join(HERE, "golden", "smsm_ranks.json")))
NB = 8


def _opts(nb, inner_max_it=20, outer=True, s=None, extra=""):
    inner = " ".join(f"-inner{b + 1}_ksp_max_it {inner_max_it} -inner{b + 1}_ksp_rtol 1e-20 -inner{b + 1}_pc_type none "
                     f"-inner{b + 1}_ksp_gmres_restart 30 -inner{b + 1}_ksp_atol 1e-100" for b in range(nb))
    out = " ".join(f"-outer{b + 1}_ksp_type lsqr -outer{b + 1}_ksp_convergence_test default "
                   f"-outer{b + 1}_ksp_lsqr_exact_mat_norm -outer{b + 1}_ksp_atol 1e-100 "
                   f"-outer{b + 1}_ksp_max_it 70 -outer{b + 1}_ksp_rtol 1e-15 -outer{b + 1}_pc_type none"
                   for b in range(nb)) if outer else ""
    return Options(f"{inner} {out} {f'-s {s}' if s else ''} {extra}")


INNER = dict(restart=30, max_it=20, rtol=1e-20, abstol=1e-100)
OUTER = dict(max_it=70, rtol=1e-15, abstol=1e-100, exact_norm=1, conv_test=0)


def _sha(x):
    return hashlib.sha256(np.ascontiguousarray(x, np.float64).tobytes()).hexdigest()


# ------------------------------------------------------------------ one process, 8 blocks
@pytest.mark.parametrize("dim,nx,ny,nz,rtol", [(3, 8, 8, 16, 1e-6), (2, 24, 32, 1, 1e-6)])
def test_sm_eight_blocks_one_process_bitwise_oracle(ctx, oracle, dim, nx, ny, nz, rtol):
    """synchronous-multisplitting.c:155-206 at nb = 8 (2 planes / 3 lines per block)."""
    comm = LocalComm()
    blocks = make_blocks(ctx, dim, nx, ny, nz, NB, range(NB), _opts(NB, outer=False), comm)
    res = sm_solve(blocks, comm, rtol=rtol, max_outer=400)
    ro = oracle.sm_solve(dim, nx, ny, nz, NB, rtol, dict(INNER, reduce_mode=oracle.REDUCE_DBR), max_outer=400)
    assert res.outer_its == ro["outer_its"] and res.norm0 == ro["norm0"]
    assert np.array_equal(np.array(res.hist), ro["hist"])
    assert np.array_equal(np.array(res.inner_its), ro["inner_its"])
    assert np.array_equal(np.concatenate([blk.x.get_array() for blk in blocks]), ro["x"])
    assert res.hist[-1] <= rtol * res.norm0


@pytest.mark.parametrize("dim,nx,ny,nz,s,rtol", [(3, 8, 8, 16, 4, 1e-6), (2, 24, 32, 1, 3, 1e-6)])
def test_smsm_eight_blocks_one_process_bitwise_oracle(ctx, oracle, dim, nx, ny, nz, s, rtol):
    """SMSM-global.c:288-363 at nb = 8: every outer LSQR residual, LSQR count and reason, every inner count,
    x and the final residual."""
    comm = LocalComm()
    blocks, mini = make_smsm(ctx, dim, nx, ny, nz, NB, range(NB), s, _opts(NB), comm)
    res = smsm_solve(blocks, comm, s, mini, rtol=rtol, max_outer=100)
    ro = oracle.smsm_solve(dim, nx, ny, nz, NB, s, rtol, dict(INNER, reduce_mode=oracle.REDUCE_DBR),
                           dict(OUTER, reduce_mode=oracle.REDUCE_DBR), max_outer=100)
    assert res.outer_its == ro["outer_its"] and res.norm0 == ro["norm0"]
    assert np.array_equal(np.array(res.hist), ro["hist"])
    assert np.array_equal(np.array(res.lsqr_its), ro["lsqr_its"])
    assert np.array_equal(np.array(res.lsqr_reason), ro["lsqr_reason"])
    assert np.array_equal(np.array(res.inner_its), ro["inner_its"])
    assert np.array_equal(np.concatenate([blk.x.get_array() for blk in blocks]), ro["x"])
    assert res.final_norm == ro["final_norm"]
    mini.close()


@pytest.mark.parametrize("variant", ["sm", "smsm"])
def test_eight_blocks_petsc_order_bitwise_oracle(oracle, variant):
    """The PETSc-order mode at nb = 8 (-msplit_reduction seq): SM and SMSM-global with 8 blocks in one process equal
    the oracle's ORC_REDUCE_SEQ bit for bit (every history entry, the inner and LSQR counts, x); the LSQR sums run
    chained across the 8 row blocks as the reference's one-rank LSQR does."""
    from medane_tchakorom_ufc_thesis_repository_amd.petsc import Context
    sctx = Context(0)
    sctx.set_reduction("seq")
    comm = LocalComm()
    dim, nx, ny, nz, s, rtol = 3, 8, 8, 16, 4, 1e-6
    if variant == "sm":
        blocks = make_blocks(sctx, dim, nx, ny, nz, NB, range(NB), _opts(NB, outer=False), comm)
        res = sm_solve(blocks, comm, rtol=rtol, max_outer=400)
        ro = oracle.sm_solve(dim, nx, ny, nz, NB, rtol, dict(INNER, reduce_mode=oracle.REDUCE_SEQ), max_outer=400)
    else:
        blocks, mini = make_smsm(sctx, dim, nx, ny, nz, NB, range(NB), s, _opts(NB), comm)
        res = smsm_solve(blocks, comm, s, mini, rtol=rtol, max_outer=100)
        ro = oracle.smsm_solve(dim, nx, ny, nz, NB, s, rtol, dict(INNER, reduce_mode=oracle.REDUCE_SEQ),
                               dict(OUTER, reduce_mode=oracle.REDUCE_SEQ), max_outer=100)
        assert np.array_equal(np.array(res.lsqr_its), ro["lsqr_its"])
        mini.close()
    assert res.outer_its == ro["outer_its"] and res.norm0 == ro["norm0"]
    assert np.array_equal(np.array(res.hist), ro["hist"])
    assert np.array_equal(np.array(res.inner_its), ro["inner_its"])
    assert np.array_equal(np.concatenate([blk.x.get_array() for blk in blocks]), ro["x"])


def _ranks_problem():
    P = RANKS["problem"]
    return P, P["nx"], P["ny"], P["planes_per_block"] * NB


def test_smsm_eight_blocks_one_process_equals_committed_record(ctx):
    """tests/golden/smsm_ranks.json['8'] (make_smsm_ranks.py, the record the driver's N = 8 bench line is checked
    against): the same 8 blocks in one process reproduce it bit for bit, block by block."""
    P, nx, ny, nz = _ranks_problem()
    rec = RANKS["worlds"][str(NB)]
    comm = LocalComm()
    blocks, mini = make_smsm(ctx, 3, nx, ny, nz, NB, range(NB), P["s"], _opts(NB), comm)
    res = smsm_solve(blocks, comm, P["s"], mini, rtol=P["rtol"], max_outer=P["outer_its"])
    mini.close()
    assert res.outer_its == rec["outer_its"] and float(res.norm0).hex() == rec["norm0_hex"]
    assert [float(h).hex() for h in res.hist] == rec["hist_hex"]
    assert [int(v) for v in res.lsqr_its] == rec["lsqr_its"]
    assert float(res.final_norm).hex() == rec["final_norm_hex"]
    assert [_sha(blk.x.get_array()) for blk in blocks] == rec["x_block_sha256"]


# ------------------------------------------------------------------ the C host, 8 MPI ranks
def _ranks_args(prog):
    P, nx, ny, nz = _ranks_problem()
    inner = [a for b in range(1, NB + 1) for a in (f"-inner{b}_ksp_max_it", "20", f"-inner{b}_ksp_rtol", "1e-20",
                                                   f"-inner{b}_ksp_atol", "1e-100")]
    outer = [a for b in range(1, NB + 1) for a in (f"-outer{b}_ksp_type", "lsqr", f"-outer{b}_ksp_convergence_test",
                                                   "default", f"-outer{b}_ksp_lsqr_exact_mat_norm",
                                                   f"-outer{b}_ksp_max_it", "70", f"-outer{b}_ksp_rtol", "1e-15",
                                                   f"-outer{b}_ksp_atol", "1e-100")]
    return [prog, "-dim", "3", "-m", str(nx), "-n", str(ny), "-p", str(nz), "-s", str(P["s"]),
            "-rtol", repr(P["rtol"]), "-max_outer", str(P["outer_its"])] + inner + outer


def _check_record(got, dump):
    rec = RANKS["worlds"][str(NB)]
    assert got["ranks"] == NB
    assert got["outer_its"] == rec["outer_its"] and float(got["norm0"]).hex() == rec["norm0_hex"]
    assert [float.fromhex(h).hex() for h in got["hist_hex"]] == rec["hist_hex"]
    assert got["lsqr_its"] == rec["lsqr_its"]
    assert float(got["final_norm"]).hex() == rec["final_norm_hex"]
    xs = [_sha(np.fromfile(f"{dump}.{b}", dtype=np.float64)) for b in range(NB)]
    assert xs == rec["x_block_sha256"]


def test_c_host_eight_mpi_ranks_host_transport_equals_record(ctx, built):
    """One block per MPI rank at 8 ranks over the host transport (MPI_Allgather through msp_comm), on the
    record's problem: outer history, LSQR counts, norm0, final residual and every rank's block of x are the
    committed 8-block oracle record's, bit for bit."""
    with tempfile.TemporaryDirectory() as d:
        dump = os.path.join(d, "x")
        got = _run(_ranks_args(SMSM) + ["-msplit_transport", "host", "-msplit_dump_x", dump], mpi=NB, timeout=240,
                   env=ONE_QUEUE)
        assert got["transport"] == "host"
        _check_record(got, dump)


def test_c_host_eight_mpi_ranks_rccl_equals_record(ctx, built):
    """The same 8 ranks over RCCL (grouped ncclSend/ncclRecv planes, ncclAllGather of the sums and LSQR partials
    on the context's stream; -msplit_require_rccl), bitwise the record."""
    with tempfile.TemporaryDirectory() as d:
        dump = os.path.join(d, "x")
        got = _run_rccl(_ranks_args(SMSM) + ["-msplit_dump_x", dump], NB, timeout=300)
        assert got["transport"] == "rccl"
        _check_record(got, dump)


def test_c_host_eight_mpi_ranks_sm_bitwise_oracle(ctx, oracle, built):
    """SM at 8 MPI ranks (host transport), 3D, to convergence: history and x bitwise the DBR oracle."""
    inner = [a for b in range(1, NB + 1) for a in (f"-inner{b}_ksp_max_it", "20", f"-inner{b}_ksp_rtol", "1e-20",
                                                   f"-inner{b}_ksp_atol", "1e-100")]
    args = [SM, "-dim", "3", "-m", "8", "-n", "8", "-p", "16", "-rtol", "1e-6"] + inner
    ro = oracle.sm_solve(3, 8, 8, 16, NB, 1e-6, dict(INNER, reduce_mode=oracle.REDUCE_DBR), max_outer=400)
    with tempfile.TemporaryDirectory() as d:
        dump = os.path.join(d, "x")
        got = _run(args + ["-msplit_transport", "host", "-msplit_dump_x", dump], mpi=NB, timeout=240, env=ONE_QUEUE)
        x = np.concatenate([np.fromfile(f"{dump}.{b}", dtype=np.float64) for b in range(NB)])
    assert got["outer_its"] == ro["outer_its"] and got["norm0"] == ro["norm0"]
    assert [float.fromhex(h) for h in got["hist_hex"]] == list(ro["hist"])
    assert np.array_equal(x, ro["x"])


# ------------------------------------------------------------------ AMAM-global, 8 blocks
PE = (0.5, 0.25, -0.3)


@pytest.mark.parametrize("minimization", ["lsqr", "rtr"])
@pytest.mark.parametrize("peclet", [None, PE], ids=["poisson", "convdiff"])
def test_amam_global_eight_blocks_roundrobin_bitwise_vs_twin(ctx, oracle, peclet, minimization):
    """AMAM-global_prime.c:371-481 at nb = 8 (configs[3] / configs[4]'s block count), round-robin in one process
    over the HBM mailboxes and the R-row (or Gram-part) broadcast: every local norm, state and phase tag of the
    trace, the counts, x, the final residual and the error are the twin's bit for bit."""
    dim, nx, ny, nz, s, max_it = 3, 8, 8, 16, 4, 5
    comm = LocalComm()
    opts = _opts(NB, inner_max_it=max_it)
    blocks = make_blocks(ctx, dim, nx, ny, nz, NB, range(NB), opts, comm, peclet)
    for blk in blocks:
        blk.setup_global_async_minimization(s, minimization=minimization)
    res = am_solve(blocks, comm, rtol=1e-6, record=True, variant="amam_global", s=s)
    tw = am_twin.amam_global_roundrobin(oracle, dim, nx, ny, nz, NB, s, 1e-6,
                                        dict(restart=30, max_it=max_it, rtol=1e-20), OUTER, peclet=peclet,
                                        minimization=minimization)
    assert res.norm0 == tw["norm0"] and res.iterations == tw["iterations"] and res.inner_its == tw["inner_its"]
    assert res.trace == tw["trace"]
    assert res.phase_tags == tw["phase_tags"]
    assert np.array_equal(np.concatenate([blk.x.get_array() for blk in blocks]), tw["x"])
    assert res.final_norm == tw["final_norm"] and res.error == tw["error"]
    last = {b: st for b, _, _, st, _ in res.trace}
    assert set(last.values()) == {ConvDetection.FINISHED} and len(last) == NB


# ------------------------------------------------------------------ configs[4] whole
C4_RTOL = 1e-4
C4_MAX_ITS = 60


def _c4_run(ctx, blocks, comm):
    for blk in blocks:                  # x = 0 and the replicated R (or Gram parts) zeroed: MatZeroEntries(R)
        blk.x.set(0.0)
        if blk.minimization == "rtr":
            for D in blk.Gc_rep:
                D.zero_entries()
        else:
            for j, D in enumerate(blk.R_rep):
                if j != blk.layout.b:
                    D.zero_entries()
    def progress(b, it, ln, st, tag):   # a line per block iteration: a long run is visibly alive (pytest -s)
        print(f"configs[4] block {b} iteration {it} local residual {ln:.3e} state {st}", flush=True)
    res = am_solve(blocks, comm, rtol=C4_RTOL, record=True, variant="amam_global", s=20, max_iterations=C4_MAX_ITS,
                   monitor=progress)
    return res, ([(b, it, float(ln).hex()) for b, it, ln, _, _ in res.trace],
                 [_sha(blk.x.get_array()) for blk in blocks], float(res.final_norm).hex())


@pytest.mark.timeout(900)
def test_configs4_whole_eight_blocks_roundrobin_rtr(ctx):
    """BASELINE configs[4] as configured: 3D upwind convection-diffusion on 512^3 in 8 z-slab blocks of
    512 x 512 x 64, AMAM-global (AMAM-global_prime.c:371-481) with s 20, inner GMRES(30) max_it 20 rtol 1e-20,
    outer LSQR max_it 70 rtol 1e-15 (running_bulk_test_g5k:296-317), -rtol 1e-4 -- all 8 blocks round-robin on
    this GPU with the normal-equations minimization (-msplit_minimization rtr: the reference's outer_solver,
    utils.c:972-996, on R^T R with Gram parts broadcast -- a mode of this library; AMAM-global itself calls
    outer_solver_norm_equation, the LSQR over the replicated R: the test below).
    The run terminates by the detection protocol (every block FINISHED in one phase, no iteration cap hit), its
    blocks passed the per-block threshold rtol/sqrt(8)*||b|| in the detection's verification, and a rerun is bitwise the first run (trace, x,
    final residual).  Asynchronous runs have no reference history."""
    comm = LocalComm()
    blocks = make_blocks(ctx, 3, 512, 512, 512, NB, range(NB),
                         _opts(NB, extra="-msplit_minimization rtr"), comm, PE)
    try:
        for blk in blocks:
            blk.setup_global_async_minimization(20)
            assert blk.minimization == "rtr"
        res, fp = _c4_run(ctx, blocks, comm)
        assert res.converged and max(res.iterations) < C4_MAX_ITS, res.iterations
        last = {b: st for b, _, _, st, _ in res.trace}
        assert last == {b: ConvDetection.FINISHED for b in range(NB)}
        assert len(set(res.phase_tags)) == 1
        assert np.isfinite(res.final_norm) and res.final_norm < res.norm0
        print(f"configs[4] whole: iterations {res.iterations}, final residual {res.final_norm:.6e} "
              f"(||b|| {res.norm0:.6e}, ratio {res.final_norm / res.norm0:.3e}), {res.elapsed:.1f} s")
        res2, fp2 = _c4_run(ctx, blocks, comm)
        assert fp2 == fp
    finally:
        del blocks
        gc.collect()


@pytest.mark.timeout(1100)
def test_configs4_whole_eight_blocks_roundrobin_lsqr(ctx):
    """BASELINE configs[4] with the minimization AMAM-global actually calls: outer_solver_norm_equation
    (AMAM-global_prime.c:425-434, utils.c:1061-1078), the LSQR over the replicated R -- every block holds all 8
    row blocks of R as last received (8 x 2.68 GB) and the global b, and publishes its own rows newest-value.
    3D upwind convection-diffusion 512^3 in 8 z-slab blocks of 512 x 512 x 64, all round-robin on this GPU (peak
    282 GB of the 309 GB HBM, tools/amam_configs.py whole: profiles/r06/configs4_lsqr/), s 20, inner GMRES(30)
    max_it 20 rtol 1e-20, outer LSQR max_it 70 rtol 1e-15, -rtol 1e-4.  The run terminates by the detection
    (every block FINISHED in one phase, no cap hit).  One run (about 100 s): the round-robin schedule's bitwise rerun
    is held by the rtr test above and, for this minimization, by tests/test_gpu_amam_configs.py's block pairs."""
    comm = LocalComm()
    blocks = make_blocks(ctx, 3, 512, 512, 512, NB, range(NB), _opts(NB, extra="-msplit_minimization lsqr"), comm,
                         PE)
    try:
        for blk in blocks:
            blk.setup_global_async_minimization(20)
            assert blk.minimization == "lsqr" and len(blk.R_rep) == NB
        res, _ = _c4_run(ctx, blocks, comm)
        assert res.converged and max(res.iterations) < C4_MAX_ITS, res.iterations
        last = {b: st for b, _, _, st, _ in res.trace}
        assert last == {b: ConvDetection.FINISHED for b in range(NB)}
        assert len(set(res.phase_tags)) == 1
        assert np.isfinite(res.final_norm) and res.final_norm < res.norm0
        print(f"configs[4] whole (lsqr): iterations {res.iterations}, final residual {res.final_norm:.6e} "
              f"(||b|| {res.norm0:.6e}, ratio {res.final_norm / res.norm0:.3e}), {res.elapsed:.1f} s, "
              f"timers {res.timers}")
    finally:
        del blocks
        gc.collect()
