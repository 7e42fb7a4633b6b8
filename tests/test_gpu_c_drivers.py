"""The C host drivers (host/: the reference's executables in C over the C ABI)
against the Python host and the oracle: same options, same outer iterations,
the same final residual to the last bit; one process (-nb blocks) and one
block per MPI rank (MPICH; both ranks share the one GPU, so the transport is
MPI_Allgather through msp_comm's host path)."""
import json
import os
import signal
import subprocess

import pytest

from medane_tchakorom_ufc_thesis_repository_amd import drivers

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOST = os.path.join(ROOT, "host")
MPIEXEC = "/opt/conda/bin/mpiexec"


@pytest.fixture(scope="module")
def built():
    subprocess.run(["make", "-s", "-C", HOST], check=True)
    return HOST


# hydra's fork launcher and the loopback interface: no ssh, no lookup of the box's hostname (a box whose name
# does not resolve would otherwise stall the PMI wire-up)
MPI_LAUNCH = ["-launcher", "fork", "-iface", "lo"]


def _run(args, mpi=0, timeout=150, env=None):
    """Run a C host driver (under mpiexec with mpi ranks); its last JSON line.  The whole process group is
    killed at the time limit (no rank is left holding the GPU) and the test fails with what it printed."""
    exe = os.path.join(HOST, "msplit_driver_mpi" if mpi else "msplit_driver")
    cmd = ([MPIEXEC] + MPI_LAUNCH + ["-n", str(mpi)] if mpi else []) + [exe] + args + ["-json"]
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, start_new_session=True,
                         env=None if env is None else {**os.environ, **env})
    try:
        out, err = p.communicate(timeout=timeout)
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, signal.SIGKILL)
        out, err = p.communicate()
        raise AssertionError(f"{' '.join(cmd)} did not finish in {timeout} s\nstdout:\n{out[-2000:]}\n"
                             f"stderr:\n{err[-2000:]}")
    assert p.returncode == 0, f"{' '.join(cmd)} exited {p.returncode}\nstderr:\n{err[-2000:]}"
    return json.loads([ln for ln in out.splitlines() if ln.startswith("{")][-1])


INNER2 = [a for b in (1, 2) for a in (f"-inner{b}_ksp_max_it", "20", f"-inner{b}_ksp_rtol", "1e-20")]
OUTER2 = [a for b in (1, 2) for a in (f"-outer{b}_ksp_type", "lsqr", f"-outer{b}_ksp_convergence_test", "default",
                                      f"-outer{b}_ksp_lsqr_exact_mat_norm", f"-outer{b}_ksp_max_it", "70",
                                      f"-outer{b}_ksp_rtol", "1e-15", f"-outer{b}_ksp_atol", "1e-100")]


@pytest.mark.parametrize("prog,args", [
    ("synchronous-multisplitting", ["-m", "32", "-n", "32", "-rtol", "1e-6"] + INNER2),
    ("synchronous-multisplitting", ["-dim", "3", "-m", "8", "-n", "8", "-p", "12", "-rtol", "1e-6",
                                    "-peclet", "0.5,0.25,-0.3"] + INNER2),
    ("synchronous-multisplitting-synchronous-minimization-global", ["-m", "32", "-n", "32", "-s", "4", "-rtol", "1e-6"]
     + INNER2 + OUTER2),
])
def test_c_host_matches_python_host(ctx, built, prog, args):
    c = _run([prog] + args)
    py = drivers.run([prog] + args + ["-json"])
    assert c["outer_its"] == py["outer_its"]
    assert c["final_norm"] == py["final_norm"] and c["error"] == py["error"]


def test_c_host_am_matches_python_host(ctx, built):
    inner = [a for b in (1, 2) for a in (f"-inner{b}_ksp_max_it", "5", f"-inner{b}_ksp_rtol", "1e-20")]
    args = ["asynchronous-multisplitting", "-dim", "3", "-m", "8", "-n", "8", "-p", "8", "-rtol", "1e-6"] + inner
    c = _run(args)
    py = drivers.run(args + ["-json"])
    assert c["iterations"] == py["iterations"]
    assert c["final_norm"] == py["final_norm"] and c["error"] == py["error"]


SM = "synchronous-multisplitting"
SMSM = "synchronous-multisplitting-synchronous-minimization-global"
INNER_ORC = dict(restart=30, max_it=20, rtol=1e-20, abstol=1e-50)
OUTER_ORC = dict(max_it=70, rtol=1e-15, abstol=1e-100, exact_norm=1, conv_test=0)


def _oracle_record(oracle, prog, dim, nx, ny, nz, nb, s, rtol):
    """The DBR oracle's run of the same problem (orc_sm_solve / orc_smsm_solve: one process, nb blocks)."""
    inner = dict(INNER_ORC, reduce_mode=oracle.REDUCE_DBR)
    if prog == SM:
        return oracle.sm_solve(dim, nx, ny, nz, nb, rtol, inner, max_outer=200)
    return oracle.smsm_solve(dim, nx, ny, nz, nb, s, rtol, inner, dict(OUTER_ORC, reduce_mode=oracle.REDUCE_DBR),
                             max_outer=200)


def _assert_same_run(got, want, what):
    """Outer count, every outer-history entry (and LSQR count), norm0 and the final residual, bit for bit; on a
    mismatch the message names the first outer iteration at which the two runs part."""
    gh = [float.fromhex(h) for h in got["hist_hex"]]
    wh = [float(v) for v in want["hist"]]
    first = next((i for i in range(min(len(gh), len(wh))) if gh[i] != wh[i]), None)
    if first is None and len(gh) != len(wh):
        first = min(len(gh), len(wh))
    detail = (f"{what}: transport {got.get('transport')}, outer_its {got['outer_its']} vs {want['outer_its']}, first "
              f"diverging outer iteration {first}\n got  hist {gh}\n want hist {wh}\n"
              f" got  lsqr {got.get('lsqr_its')}\n want lsqr {list(want.get('lsqr_its', []))}")
    assert first is None and got["outer_its"] == want["outer_its"], detail
    if "lsqr_its" in want:
        assert got["lsqr_its"] == [int(v) for v in want["lsqr_its"]], detail
    assert got["norm0"] == want["norm0"], detail


def _problem_args(prog, dim, nx, ny, nz, nb, s, rtol):
    a = ["-m", str(nx), "-n", str(ny), "-rtol", repr(rtol)] + _inner(nb, 20)
    if dim == 3:
        a = ["-dim", "3", "-p", str(nz)] + a
    if prog == SMSM:
        a += ["-s", str(s)] + _outer(nb)
    return [prog] + a


# SM and SMSM-global at 2, 3 and 4 ranks, 2D and 3D (24 lines of 32 / 12 planes divide by every world size).  The
# 3D 8x8x8 SMSM-global case is the one GPUTEST_r03 caught at 5 outer iterations against the oracle's 3.
MPI_CASES = [(SM, 2, 24, 32, 1, 2, 0, 1e-6), (SMSM, 3, 8, 8, 8, 2, 4, 1e-6),
             (SMSM, 2, 24, 32, 1, 2, 4, 1e-6), (SM, 3, 8, 8, 12, 3, 0, 1e-6), (SMSM, 3, 8, 8, 12, 3, 4, 1e-6),
             (SMSM, 2, 24, 32, 1, 3, 3, 1e-6), (SM, 2, 24, 32, 1, 4, 0, 1e-6), (SMSM, 3, 8, 8, 12, 4, 4, 1e-6)]


@pytest.mark.parametrize("case", MPI_CASES, ids=lambda c: f"{'smsm' if c[0] == SMSM else 'sm'}-{c[1]}d-{c[5]}ranks")
def test_c_host_mpi_ranks_equal_oracle(ctx, oracle, built, case):
    """One block per MPI rank over the host transport (every rank shares the box's one GPU, which RCCL refuses;
    pinned with -msplit_transport host so the run says which transport it took): the outer history, the LSQR
    counts and the final residual are the single-process run's and the DBR oracle's, bit for bit
    (comm.c:126-141, synchronous-multisplitting.c:170-206, SMSM-global.c:288-363)."""
    prog, dim, nx, ny, nz, nb, s, rtol = case
    args = _problem_args(prog, dim, nx, ny, nz, nb, s, rtol)
    want = _oracle_record(oracle, prog, dim, nx, ny, nz, nb, s, rtol)
    one = _run(args + ["-nb", str(nb)])
    _assert_same_run(one, want, "one process vs oracle")
    got = _run(args + ["-msplit_transport", "host"], mpi=nb)
    assert got["ranks"] == nb and got["transport"] == "host"
    _assert_same_run(got, want, f"{nb} MPI ranks vs oracle")
    assert got["final_norm"] == one["final_norm"] and got["error"] == one["error"]
    if prog == SMSM:
        assert got["final_norm"] == want["final_norm"]


@pytest.mark.parametrize("case", [MPI_CASES[1], MPI_CASES[6]], ids=["smsm-3d-2ranks", "sm-2d-4ranks"])
def test_c_host_mpi_serialized_equals_oracle(ctx, oracle, built, case):
    """The same multi-rank runs with every kernel and copy serialised by the HIP runtime (AMD_SERIALIZE_KERNEL=3,
    AMD_SERIALIZE_COPY=3).  Before round 4's fix the host-transport exchange and ordered sum staged through
    hipMallocAsync/hipFreeAsync blocks that were reused while a copy was still in flight.  Under serialisation that
    failed every case from the first outer iteration: this 3D SMSM-global case gave r03's 5 outer iterations
    against the oracle's 3 (profiles/r04/comm_fix/).  A result that depends on how the runtime overlaps copies and
    kernels fails here."""
    prog, dim, nx, ny, nz, nb, s, rtol = case
    args = _problem_args(prog, dim, nx, ny, nz, nb, s, rtol)
    want = _oracle_record(oracle, prog, dim, nx, ny, nz, nb, s, rtol)
    got = _run(args + ["-msplit_transport", "host"], mpi=nb, env={"AMD_SERIALIZE_KERNEL": "3", "AMD_SERIALIZE_COPY": "3"})
    assert got["ranks"] == nb and got["transport"] == "host"
    _assert_same_run(got, want, f"{nb} MPI ranks, serialised, vs oracle")


# RCCL refuses two ranks of one host on one GPU ("Duplicate GPU detected").  With a different NCCL_HOSTID per rank it
# takes them for separate hosts and connects them over its socket transport on the loopback interface: not xGMI,
# but msplit_comm.hip's RCCL branch -- grouped ncclSend/ncclRecv of the planes, ncclAllGather of the ordered sums and
# LSQR partials, all on the context's stream -- runs multi-rank on this one-GPU box.
RCCL_ENV = ["-env", "NCCL_SOCKET_IFNAME", "lo", "-env", "NCCL_IB_DISABLE", "1"]


def _run_rccl(args, nranks, timeout=150):
    """One rank per block over RCCL (MPMD launch, one NCCL_HOSTID per rank), -msplit_require_rccl: the run stops
    rather than fall back to the host transport.  Its last JSON line."""
    exe = os.path.join(HOST, "msplit_driver_mpi")
    cmd = [MPIEXEC] + MPI_LAUNCH
    for r in range(nranks):
        cmd += (([":"] if r else []) + ["-n", "1"] + RCCL_ENV + ["-env", "NCCL_HOSTID", f"msplit-test-rank{r}", exe]
                + args + ["-msplit_require_rccl", "-json"])
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, start_new_session=True)
    try:
        out, err = p.communicate(timeout=timeout)
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, signal.SIGKILL)
        out, err = p.communicate()
        raise AssertionError(f"RCCL run did not finish in {timeout} s\nstderr:\n{err[-3000:]}")
    assert p.returncode == 0, f"RCCL run exited {p.returncode}\nstderr:\n{err[-3000:]}"
    return json.loads([ln for ln in out.splitlines() if ln.startswith("{")][-1])


@pytest.mark.parametrize("case", [MPI_CASES[1], MPI_CASES[0], MPI_CASES[4], MPI_CASES[6], MPI_CASES[7]],
                         ids=lambda c: f"{'smsm' if c[0] == SMSM else 'sm'}-{c[1]}d-{c[5]}ranks")
def test_c_host_mpi_rccl_ranks_equal_oracle(ctx, oracle, built, case):
    """The RCCL transport multi-rank (the N > 1 product path; on this box over RCCL's socket transport, see
    RCCL_ENV): SM and SMSM-global at 2, 3 and 4 ranks, bitwise the DBR oracle and the host-transport run --
    outer history, LSQR counts, norm0, final residual and error (comm.c:126-141, :252-286)."""
    prog, dim, nx, ny, nz, nb, s, rtol = case
    args = _problem_args(prog, dim, nx, ny, nz, nb, s, rtol)
    want = _oracle_record(oracle, prog, dim, nx, ny, nz, nb, s, rtol)
    got = _run_rccl(args, nb)
    assert got["ranks"] == nb and got["transport"] == "rccl"
    _assert_same_run(got, want, f"{nb} MPI ranks over RCCL vs oracle")
    host = _run(args + ["-msplit_transport", "host"], mpi=nb)
    assert got["final_norm"] == host["final_norm"] and got["error"] == host["error"]
    if prog == SMSM:
        assert got["final_norm"] == want["final_norm"]


def test_c_host_mpi_require_rccl_refuses_the_host_path(built):
    """-msplit_require_rccl: two ranks on one GPU cannot get an RCCL communicator, so the run stops (exit 3)
    before any solve instead of silently measuring the MPI path."""
    exe = os.path.join(HOST, "msplit_driver_mpi")
    p = subprocess.run([MPIEXEC] + MPI_LAUNCH + ["-n", "2", exe] + _problem_args(SM, 2, 24, 32, 1, 2, 0, 1e-6)
                       + ["-msplit_require_rccl", "-json"], capture_output=True, text=True, timeout=150)
    assert p.returncode != 0 and "require_rccl" in p.stderr
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]


def test_c_host_mpi_am_terminates(ctx, built):
    inner = [a for b in (1, 2) for a in (f"-inner{b}_ksp_max_it", "5", f"-inner{b}_ksp_rtol", "1e-20")]
    r = _run(["asynchronous-multisplitting", "-dim", "3", "-m", "8", "-n", "8", "-p", "16", "-rtol", "1e-6"] + inner,
             mpi=2)
    assert len(r["iterations"]) == 1 and r["final_norm"] < 1e-4 * r["norm0"]


def _inner(nb, its):
    return [a for b in range(1, nb + 1) for a in (f"-inner{b}_ksp_max_it", str(its), f"-inner{b}_ksp_rtol", "1e-20")]


def _outer(nb):
    return [a for b in range(1, nb + 1) for a in (f"-outer{b}_ksp_type", "lsqr", f"-outer{b}_ksp_convergence_test",
                                                  "default", f"-outer{b}_ksp_lsqr_exact_mat_norm",
                                                  f"-outer{b}_ksp_max_it", "70", f"-outer{b}_ksp_rtol", "1e-15",
                                                  f"-outer{b}_ksp_atol", "1e-100")]


AMAM = "asynchronous-multisplitting-asynchronous-minimization-global"


@pytest.mark.parametrize("args", [
    ["-dim", "3", "-m", "8", "-n", "8", "-p", "8", "-s", "4", "-rtol", "1e-6"] + _inner(2, 5) + _outer(2),
    ["-m", "32", "-n", "32", "-s", "3", "-rtol", "1e-6"] + _inner(2, 8) + _outer(2),
    ["-dim", "3", "-m", "8", "-n", "8", "-p", "12", "-nb", "3", "-s", "4", "-rtol", "1e-6",
     "-peclet", "0.5,0.25,-0.3"] + _inner(3, 5) + _outer(3),
])
@pytest.mark.parametrize("minimization", ["lsqr", "rtr"])
def test_c_host_amam_global_matches_python_host(ctx, built, args, minimization):
    """AMAM-global (configs[3]/[4]'s algorithm) in the C host, blocks round-robin in one process: the same
    per-block iteration counts, final residual and error as the Python host, to the last bit; with the
    replicated-R LSQR and with the reference's outer_solver (-msplit_minimization rtr)."""
    args = args + ["-msplit_minimization", minimization]
    c = _run([AMAM] + args)
    py = drivers.run([AMAM] + args + ["-json"])
    assert c["iterations"] == py["iterations"]
    assert c["final_norm"] == py["final_norm"] and c["error"] == py["error"]


@pytest.mark.parametrize("minimization", ["lsqr", "rtr"])
def test_c_host_mpi_amam_global_terminates(ctx, built, minimization):
    """One block per MPI rank (both on the one GPU): the R rows (or Gram parts) travel between the processes' HBM
    through the msp_abcast buffers, the detection ends the run, and the residual meets the tolerance."""
    r = _run([AMAM, "-dim", "3", "-m", "8", "-n", "8", "-p", "16", "-s", "4", "-rtol", "1e-6",
              "-msplit_minimization", minimization] + _inner(2, 5) + _outer(2), mpi=2)
    assert len(r["iterations"]) == 1 and r["final_norm"] < 1e-4 * r["norm0"]


@pytest.mark.parametrize("reduction", ["seq", "dbr"])
def test_c_host_configs0_reduction_option_matches_oracle(ctx, oracle, built, reduction):
    """BASELINE configs[0] (2D 256^2, SMSM-global, 2 blocks, s 4, rtol 1e-3, the campaign's inner/outer options)
    from the reference's own command line on the C host.  -msplit_reduction seq (the parity mode) reproduces the
    PETSc-order oracle's first 20 outer iterations bit for bit -- outer count, every outer LSQR residual norm,
    every LSQR iteration count, and the final residual; -msplit_reduction dbr (the default) the DBR oracle's."""
    cap = 20
    inner = [a for b in (1, 2) for a in (f"-inner{b}_ksp_max_it", "20", f"-inner{b}_ksp_rtol", "1e-3",
                                         f"-inner{b}_ksp_gmres_restart", "30", f"-inner{b}_pc_type", "none")]
    args = (["synchronous-multisplitting-synchronous-minimization-global", "-m", "256", "-n", "256", "-s", "4",
             "-rtol", "1e-3", "-nb", "2", "-max_outer", str(cap), "-msplit_reduction", reduction] + inner + OUTER2)
    c = _run(args)
    mode = oracle.REDUCE_SEQ if reduction == "seq" else oracle.REDUCE_DBR
    ro = oracle.smsm_solve(2, 256, 256, 1, 2, 4, 1e-3, dict(restart=30, max_it=20, rtol=1e-3, abstol=1e-50,
                                                            reduce_mode=mode),
                           dict(max_it=70, rtol=1e-15, abstol=1e-100, exact_norm=1, conv_test=0, reduce_mode=mode),
                           max_outer=cap)
    assert c["outer_its"] == ro["outer_its"]
    assert [float.fromhex(h) for h in c["hist_hex"]] == list(ro["hist"])
    assert c["lsqr_its"] == list(ro["lsqr_its"])
    assert c["norm0"] == ro["norm0"] and c["final_norm"] == ro["final_norm"]
    if reduction == "seq":
        assert c["outer_its"] == cap        # the PETSc-order run stagnates just above 1e-3
    py = drivers.run(args + ["-json"])    # the Python host takes the same option
    assert py["outer_its"] == c["outer_its"] and py["hist"] == list(ro["hist"])


ISOLVE_CONFIGS0 = ["--np", "2", "--npb", "1", "--m", "256", "--n", "256", "--s", "4", "--rtol", "1e-3",
                   "--alg", "SMSM_GLOBAL", "--inner-ksp", "gmres", "--inner-rtol", "1e-3", "--inner-max-iters", "20",
                   "--inner-pc-type", "none", "--outer-ksp", "lsqr", "--outer-rtol", "1e-15",
                   "--outer-max-iters", "70", "--outer-pc-type", "none", "--other-petsc-options",
                   "-inner_ksp_gmres_restart 30 -outer_ksp_convergence_test default -outer_ksp_lsqr_exact_mat_norm "
                   "-outer_ksp_atol 1e-100 -json"]


def _isolve(args, launch):
    env = dict(os.environ, ISOLVE_LAUNCH=launch)
    p = subprocess.run([os.path.join(HOST, "isolve")] + args, capture_output=True, text=True, env=env, timeout=300,
                       start_new_session=True)
    assert p.returncode == 0, p.stderr[-3000:]
    return json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])


@pytest.mark.parametrize("launch", ["single", "mpi"])
def test_isolve_configs0_command_line_equals_explicit_prefixes_and_oracle(ctx, oracle, built, launch):
    """BASELINE configs[0] as an iSolve command line (iSolve:118-194; --np 2 --alg SMSM_GLOBAL, the campaign's
    inner/outer options, running_bulk_test_g5k:247-248) through host/isolve: the run is the explicit-prefix C-host
    run (-inner1_/-inner2_/-outer1_/-outer2_) and the DBR oracle, bit for bit -- outer count, every outer LSQR
    residual and LSQR count, the final residual -- in one process (-nb 2) and over 2 MPI ranks."""
    got = _isolve(ISOLVE_CONFIGS0, launch)
    inner = [a for b in (1, 2) for a in (f"-inner{b}_ksp_type", "gmres", f"-inner{b}_ksp_max_it", "20",
                                         f"-inner{b}_ksp_rtol", "1e-3", f"-inner{b}_ksp_gmres_restart", "30",
                                         f"-inner{b}_pc_type", "none")]
    explicit = _run([SMSM, "-m", "256", "-n", "256", "-s", "4", "-rtol", "1e-3", "-nb", "2"] + inner + OUTER2)
    assert got["transport"] == ("host" if launch == "mpi" else "none") and got["ranks"] == (2 if launch == "mpi" else 1)
    assert got["hist_hex"] == explicit["hist_hex"] and got["lsqr_its"] == explicit["lsqr_its"]
    assert got["outer_its"] == explicit["outer_its"] and got["final_norm"] == explicit["final_norm"]
    ro = oracle.smsm_solve(2, 256, 256, 1, 2, 4, 1e-3,
                           dict(restart=30, max_it=20, rtol=1e-3, abstol=1e-50, reduce_mode=oracle.REDUCE_DBR),
                           dict(OUTER_ORC, reduce_mode=oracle.REDUCE_DBR), max_outer=200)
    _assert_same_run(got, ro, f"isolve configs[0] ({launch})")
    assert got["final_norm"] == ro["final_norm"]


@pytest.mark.parametrize("prog", [SM, SMSM])
def test_c_host_mpi_stop_disagreement_exits_instead_of_hanging(built, prog):
    """Every rank agrees on (outer iteration, stop) once per outer iteration through msp_comm_agree.  With rank 1
    injected to stop alone at the first outer iteration (MSPLIT_FAULT_STOP_RANK=1), the run exits non-zero on
    every rank within seconds, naming the disagreement -- round 4's pre-fix corruption hung such a run until its
    150 s limit (profiles/r04/comm_fix/)."""
    exe = os.path.join(HOST, "msplit_driver_mpi")
    args = _problem_args(prog, 3, 8, 8, 12, 2, 4, 1e-6)
    p = subprocess.run([MPIEXEC] + MPI_LAUNCH + ["-n", "2", "-env", "MSPLIT_FAULT_STOP_RANK", "1", exe] + args
                       + ["-msplit_transport", "host", "-json"], capture_output=True, text=True, timeout=120,
                       start_new_session=True)
    assert p.returncode != 0
    assert "disagree" in p.stderr, p.stderr[-2000:]
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]


AM = "asynchronous-multisplitting"
PE3 = ["-peclet", "0.5,0.25,-0.3"]


@pytest.mark.parametrize("prog,extra,nbuf", [
    (AM, [], "2"),
    (AM, PE3, "2"),
    (AMAM, ["-msplit_minimization", "lsqr"], "2"),
    (AMAM, ["-msplit_minimization", "lsqr"], "1"),
    (AMAM, ["-msplit_minimization", "lsqr"] + PE3, "1"),
    (AMAM, ["-msplit_minimization", "rtr"], "2"),
    (AMAM, ["-msplit_minimization", "rtr"] + PE3, "1"),
], ids=["am", "am-convdiff", "amam-lsqr-nbuf2", "amam-lsqr-nbuf1", "amam-lsqr-convdiff-nbuf1", "amam-rtr-nbuf2",
        "amam-rtr-convdiff-nbuf1"])
def test_c_host_eight_mpi_ranks_async_terminates(ctx, built, prog, extra, nbuf):
    """configs[3]/[4]'s world size on the C host: 8 MPI ranks, one block each, truly asynchronous on the one GPU
    (planes, and the R rows or Gram parts, through HBM slots opened by IPC; the detection over a chain of
    diameter 7: conv_detection_prime.c:11-210, AMAM-global_prime.c:371-481).  Every rank's own report (gathered on
    rank 0): FINISHED, one phase tag, the same global final residual below the threshold, the drain of the pending
    messages and the completion of the sends still in flight done (comm.c:426-453, AMAM-global_prime.c:522-572),
    and the run exits 0."""
    args = [prog, "-dim", "3", "-m", "8", "-n", "8", "-p", "32", "-rtol", "1e-6", "-msplit_transport", "host"]
    args += _inner(8, 5) + (["-s", "4"] + _outer(8) if prog == AMAM else []) + extra
    r = _run(args, mpi=8, timeout=300, env={"MSPLIT_ABCAST_NBUF": nbuf, "GPU_MAX_HW_QUEUES": "1"})  # see
    # tests/test_gpu_async_mp.py: eight ranks plus this GPU-using parent must stay within the 24 compute-queue slots
    rep = r["blocks_report"]
    assert r["ranks"] == 8 and [q["block"] for q in rep] == list(range(8))
    assert all(q["state"] == 3 for q in rep), rep                       # MSP_CVD_FINISHED
    assert len({q["tag"] for q in rep}) == 1, rep
    assert all(q["final_norm"] == r["final_norm"] and q["error"] == r["error"] for q in rep)
    assert r["final_norm"] <= 1e-4 * r["norm0"]
    assert all(q["discarded"] >= 0 and q["in_flight"] >= 0 for q in rep)
    print("iterations", [q["iterations"] for q in rep], "discarded", [q["discarded"] for q in rep],
          "in_flight", [q["in_flight"] for q in rep])
