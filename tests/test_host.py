"""CPU tests of the boundary and the host logic (no compute calls)."""
import glob
import os
import subprocess
import sys

import numpy as np
import pytest

from medane_tchakorom_ufc_thesis_repository_amd import _lib, utils
from medane_tchakorom_ufc_thesis_repository_amd.petsc import Options

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_loads_and_exports_every_header_symbol():
    L = _lib.load()
    syms = _lib.header_symbols()
    assert len(syms) > 40
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing
    # the dynamic symbol table of the .so, independently of ctypes
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if " T " in ln}
    assert set(syms) <= exported, sorted(set(syms) - exported)
    # every header symbol has a binding signature
    assert set(syms) == set(_lib._SIGS) | {"msp_get_last_error", "msp_build_source_digest"}


def test_library_built_from_this_tree():
    """The .so in the tree was compiled from the sources in the tree (csrc/Makefile's digest of them), so every
    GPU result is evidence for these sources and not for a stale build."""
    assert _lib.build_digest() == _lib.source_digest(), \
        "libmsplit_hip.so is stale: rebuild with `python -c 'import __graft_entry__ as g; g.build()'`"


def test_library_is_gfx950_code():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-n", _lib.LIB_PATH], capture_output=True,
                         text=True)
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_no_gpu_means_loud_failure():
    """Without a GPU the product path raises; there is no CPU fallback."""
    from medane_tchakorom_ufc_thesis_repository_amd.petsc import Context, device_count
    if device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(_lib.MsplitError):
        Context(0)


def test_options_database_prefixes():
    o = Options("-m 256 -n 128 -rtol 1e-3 -inner1_ksp_max_it 20 -inner1_ksp_rtol 1e-20 -inner2_pc_type none "
                "-ksp_converged_use_initial_residual_norm -x -1.5")
    assert o.get_int("m") == 256 and o.get_int("n") == 128
    assert o.get_real("rtol") == 1e-3
    assert o.get_int("ksp_max_it", prefix="inner1_") == 20
    assert o.get_real("ksp_rtol", prefix="inner1_") == 1e-20
    assert o.get_int("ksp_max_it", 10000, prefix="inner2_") == 10000
    assert o.get_string("pc_type", prefix="inner2_") == "none"
    assert o.get_bool("ksp_converged_use_initial_residual_norm")
    assert o.get_real("x") == -1.5


def _dense_block(L, A_rows):
    rp, c, v, nc = A_rows
    D = np.zeros((rp.size - 1, nc))
    for r in range(rp.size - 1):
        D[r, c[rp[r]:rp[r + 1]]] = v[rp[r]:rp[r + 1]]
    return D


@pytest.mark.parametrize("dim,nx,ny,nz,nb", [(3, 5, 4, 6, 3), (3, 4, 3, 4, 4), (3, 3, 3, 2, 1),
                                             (2, 8, 6, 1, 4), (2, 6, 5, 1, 2)])
def test_block_layout_reproduces_the_split(dim, nx, ny, nz, nb):
    """A_ii (box stencil) + coupling rows in halo numbering == the host split of
    the reference's block rows (divideSubDomainIntoBlockMatrices)."""
    for b in range(nb):
        L = utils.block_layout(dim, nx, ny, nz, nb, b)
        if dim == 3:
            rows = utils.poisson3DMatrix_rows(nx, ny, nz, b * nz // nb, (b + 1) * nz // nb)
        else:
            rows = utils.poisson2DMatrix_rows(nx, ny, L.r0, L.r1)
        (rpi, ci, vi), (rpo, co, vo) = utils.split_columns(*rows[:3], L.r0, L.r1)
        bd, bx, by, bz = L.box
        if bd == 3:
            box = utils.poisson3DMatrix_rows(bx, by, bz, 0, bz)
        else:
            box = utils.poisson2DMatrix_rows(by, bx, 0, bx * by)
        assert np.array_equal(box[0], rpi) and np.array_equal(box[1], ci) and np.array_equal(box[2], vi)
        # coupling: map halo index back to the global column it stands for
        halo_global = np.zeros(L.halo_size, np.int64)
        for nbr, hoff, cnt, nbr_off in L.recv:
            nbr_r0 = utils.block_layout(dim, nx, ny, nz, nb, nbr).r0
            halo_global[hoff:hoff + cnt] = nbr_r0 + nbr_off + np.arange(cnt)
        row_ids, crp, cc, cv = L.coupling
        full_rp = np.zeros(L.nrows + 1, np.int64)
        full_rp[row_ids + 1] = np.diff(crp)
        full_rp = np.cumsum(full_rp)
        assert np.array_equal(full_rp, rpo)
        assert np.array_equal(halo_global[cc], co) and np.array_equal(cv, vo)
        # what I send is exactly what my neighbours' halos expect
        for nbr, off, cnt in L.send:
            Ln = utils.block_layout(dim, nx, ny, nz, nb, nbr)
            (match,) = [r for r in Ln.recv if r[0] == b]
            assert match[2] == cnt and match[3] == off


def test_oracle_is_not_imported_by_the_product():
    """The product package never references the oracle."""
    pkg = os.path.join(ROOT, "medane_tchakorom_ufc_thesis_repository_amd")
    for dp, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".c", ".hip", ".h", ".cpp")):
                txt = open(os.path.join(dp, f)).read()
                assert "pyoracle" not in txt and "liborc" not in txt and "oracle.h" not in txt, f


def test_drivers_command_line():
    """The reference executables' names and options (PetscOptionsGet* in each driver's main)."""
    from medane_tchakorom_ufc_thesis_repository_amd import drivers
    prog, opts, p = drivers.parse(["synchronous-multisplitting-synchronous-minimization-global", "-m", "64", "-n",
                                   "32", "-s", "4", "-rtol", "1e-3", "-inner1_ksp_max_it", "20", "-npb", "1"])
    assert prog.endswith("global") and (p["m"], p["n"], p["s"], p["rtol"], p["dim"]) == (64, 32, 4, 1e-3, 2)
    assert opts.get_int("ksp_max_it", prefix="inner1_") == 20
    p = drivers.parse(["asynchronous-multisplitting", "-dim", "3", "-m", "8", "-n", "8", "-peclet", "0.5,0,0"])[2]
    assert p["p"] == 8 and p["peclet"] == (0.5, 0.0, 0.0)
    for bad in (["nope"], ["synchronous-multisplitting", "-npb", "2"], ["gmres_solution", "-dim", "4"],
                ["asynchronous-multisplitting", "-peclet", "1,2"]):
        with pytest.raises(ValueError):
            drivers.parse(bad)
    assert len(drivers.PROGRAMS) == 9                                 # every driver directory of the reference's src/


def test_bench_cpu_share_and_topology(monkeypatch):
    """bench.py's CPU baseline uses the job's CPU share: MSPLIT_CPU_THREADS, else the cgroup quota / CPU set,
    capped by OMP_NUM_THREADS; the topology it reports has the fields the JSON promises."""
    import importlib
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    bench = importlib.import_module("bench")
    topo = bench.host_topology()
    assert topo["nproc"] == os.cpu_count()
    monkeypatch.delenv("MSPLIT_CPU_THREADS", raising=False)
    monkeypatch.setenv("OMP_NUM_THREADS", "3")
    assert bench.cpu_threads({"cgroup_cpu_quota": 16.0, "nproc": 256}) == 3
    monkeypatch.delenv("OMP_NUM_THREADS")
    assert bench.cpu_threads({"cgroup_cpu_quota": 16.0, "nproc": 256}) == 16
    assert bench.cpu_threads({"affinity_cpus": 8, "nproc": 256}) == 8
    monkeypatch.setenv("MSPLIT_CPU_THREADS", "5")
    assert bench.cpu_threads({"cgroup_cpu_quota": 16.0}) == 5


def test_bench_reads_the_measured_streaming_ceiling():
    """The roofline's measured ceiling comes from the committed stream_ceiling record (profiles/r03/); the rates
    are in TB/s, below the 8 TB/s spec, reading at least as fast as the MAXPY mix."""
    import importlib
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    bench = importlib.import_module("bench")
    c = bench.load_ceiling()
    assert c is not None and c["source"].startswith("profiles/r03/stream_ceiling/")
    assert 5.0 < c["maxpy_mix_TBps"] <= c["read_TBps"] < bench.HBM_PEAK_GBS / 1e3
    assert 5.0 < c["copy_TBps"] < bench.HBM_PEAK_GBS / 1e3


def test_bench_smsm_seq_line_reads_its_record():
    """bench.py's smsm_seq_mode line (in every N = 1 run; --no-seq-smsm skips it) checks the fields of
    tests/golden/smsm_seq.json that smsm_solve reports, at the block and options the record names."""
    import importlib
    import json
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    bench = importlib.import_module("bench")
    g = json.load(open(bench.SMSM_SEQ_GOLDEN))
    assert {"outer_its", "norm0_hex", "hist_hex", "lsqr_its", "inner_its", "x_sha256"} <= set(g)
    assert g["problem"]["nb"] == 1 and g["inner"]["restart"] == 30 and g["outer"]["max_it"] == 70
    old = sys.argv
    try:
        sys.argv = ["bench.py", "--no-seq-smsm"]
        assert bench.parse().no_seq_smsm
        sys.argv = ["bench.py"]
        assert not bench.parse().no_seq_smsm
    finally:
        sys.argv = old


def _isolve(args, **env):
    e = dict(os.environ, ISOLVE_DRYRUN="1", **env)
    p = subprocess.run([os.path.join(ROOT, "host", "isolve")] + args, capture_output=True, text=True, env=e,
                       timeout=60)
    assert p.returncode == 0, p.stderr
    return p.stdout.splitlines()


def test_isolve_maps_every_flag_onto_every_block_prefix():
    """host/isolve takes iSolve's command line (iSolve:118-194) and, unlike the reference -- whose drivers read
    inner1_/inner2_ while iSolve writes inner_ (iSolve:349-371, default_run_variables:54,68) -- sets every
    --inner-* / --outer-* flag and every -inner_* / -outer_* option on each block's prefix."""
    cmd = _isolve(["--np", "3", "--m", "24", "--n", "32", "--s", "5", "--rtol", "1e-4", "--alg", "SMSM_GLOBAL",
                   "--inner-ksp", "gmres", "--inner-rtol", "1e-20", "--inner-max-iters", "20", "--inner-pc-type",
                   "none", "--outer-ksp", "lsqr", "--outer-rtol", "1e-15", "--outer-max-iters", "70",
                   "--outer-pc-type", "none", "--other-petsc-options",
                   "-inner_ksp_gmres_restart 30 -outer_ksp_lsqr_exact_mat_norm -outer_ksp_convergence_test default "
                   "-json"])
    assert cmd[cmd.index("-n") + 1] == "3" and cmd[cmd.index("-n") + 2].endswith("host/msplit_driver_mpi")
    assert "synchronous-multisplitting-synchronous-minimization-global" in cmd

    def opt(k):
        i = cmd.index(k)
        return cmd[i + 1] if i + 1 < len(cmd) and not cmd[i + 1].startswith("-") else True
    for b in (1, 2, 3):
        assert opt(f"-inner{b}_ksp_type") == "gmres" and opt(f"-inner{b}_ksp_rtol") == "1e-20"
        assert opt(f"-inner{b}_ksp_max_it") == "20" and opt(f"-inner{b}_pc_type") == "none"
        assert opt(f"-inner{b}_ksp_gmres_restart") == "30"
        assert opt(f"-outer{b}_ksp_type") == "lsqr" and opt(f"-outer{b}_ksp_max_it") == "70"
        assert opt(f"-outer{b}_ksp_lsqr_exact_mat_norm") is True
        assert opt(f"-outer{b}_ksp_convergence_test") == "default"
    assert opt("-s") == "5" and opt("-rtol") == "1e-4" and opt("-m") == "24" and "-json" in cmd
    assert not any(c.startswith("-inner_") or c.startswith("-outer_") for c in cmd)


def test_isolve_single_process_and_python_variants():
    cmd = _isolve(["--np", "2", "--alg", "SM"], ISOLVE_LAUNCH="single")
    assert cmd[0].endswith("host/msplit_driver") and cmd[cmd.index("-nb") + 1] == "2"
    assert not any(c.startswith("-outer") for c in cmd) and "-s" not in cmd
    cmd = _isolve(["--np", "4", "--alg", "AMAM_SEMI_LOCAL", "--outer-ksp", "lsqr"])
    assert cmd[:3] == ["python3", "-m", "medane_tchakorom_ufc_thesis_repository_amd.drivers"]
    assert cmd[3] == "asynchronous-multisplitting-asynchronous-minimization-semi-local"   # iSolve:56 runs the -local binary
    assert cmd[cmd.index("-nb") + 1] == "4" and cmd[cmd.index("-outer4_ksp_type") + 1] == "lsqr"
    p = subprocess.run([os.path.join(ROOT, "host", "isolve"), "--np", "2", "--npb", "2"], capture_output=True,
                       text=True, env=dict(os.environ, ISOLVE_DRYRUN="1"), timeout=60)
    assert p.returncode != 0 and "npb" in p.stderr


def _split_top(args: str):
    """The comma-separated items of an argument or parameter list, at parenthesis depth 0."""
    items, depth, cur = [], 0, ""
    for ch in args:
        if ch in "([{":
            depth += 1
        elif ch in ")]}":
            depth -= 1
        if ch == "," and depth == 0:
            items.append(cur)
            cur = ""
        else:
            cur += ch
    if cur.strip():
        items.append(cur)
    return [i.strip() for i in items]


def _header_arity():
    import re
    txt = open(os.path.join(ROOT, "include", "msplit.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    out = {}
    for m in re.finditer(r"\b(?:int\s+|const char\s*\*\s*|void\s+)(msp_\w+)\s*\(([^;{]*?)\)\s*;", txt, flags=re.S):
        params = _split_top(m.group(2))
        out[m.group(1)] = 0 if params in ([], ["void"]) else len(params)
    return out


def _calls(src: str):
    """(name, argument count, line) of every msp_* call in a C source."""
    import re
    src = re.sub(r"/\*.*?\*/", lambda m: "\n" * m.group(0).count("\n"), src, flags=re.S)
    for m in re.finditer(r"\b(msp_\w+)\s*\(", src):
        i, depth = m.end(), 1
        while depth:
            depth += {"(": 1, ")": -1}.get(src[i], 0)
            i += 1
        yield m.group(1), len(_split_top(src[m.end():i - 1])), src.count("\n", 0, m.start()) + 1


def test_plugin_calls_match_the_c_abi():
    """plugin/petsc/*.c cannot be compiled here (no PETSc in the image), so its use of the C ABI is checked as text:
    every msp_* function it calls is declared in include/msplit.h and called with the declared argument count."""
    decl = _header_arity()
    assert len(decl) > 80
    seen = 0
    for fn in glob.glob(os.path.join(ROOT, "plugin", "petsc", "*.c")):
        for name, nargs, line in _calls(open(fn).read()):
            assert name in decl, f"{os.path.basename(fn)}:{line}: {name} is not declared in include/msplit.h"
            assert nargs == decl[name], (f"{os.path.basename(fn)}:{line}: {name} called with {nargs} arguments, "
                                         f"declared with {decl[name]}")
            seen += 1
    assert seen > 40


def test_plugin_device_choice_is_not_collective_per_object():
    """The node-local rank is found once, in the registration every rank runs inside PetscInitialize; the
    per-object paths (each block's KSPSetUp, the first VECMSPLIT) never call a collective."""
    src = open(os.path.join(ROOT, "plugin", "petsc", "petsc_msplit_ksp.c")).read()
    body = src[src.index("PetscErrorCode MSplitDefaultDevice(int *dev)"):]
    body = body[:body.index("\n}\n")]
    assert "MPI_Comm_split_type" not in body and "MPI_" not in body
    reg = src[src.index("PetscErrorCode MSplitRegisterAll(void)"):]
    assert "MSplitCacheLocalRank()" in reg[:reg.index("\n}\n")]


def test_plugin_ksp_reduction_does_not_leak_into_the_shared_context():
    """msplitgmres / msplitlsqr share the process's one context with VECMSPLIT and aijmsplit, whose
    order is the global -msplit_reduction.  A KSP's own (prefixed) -msplit_reduction is applied only around its
    solve: both KSPSolve entries go through MSplitSolveInOrder, which restores the context's order on every exit,
    and no other plugin code sets the order except the global option (petsc_msplit_vecmat.c).  PETSc is absent,
    so the plugin is checked as source."""
    import re
    src = open(os.path.join(ROOT, "plugin", "petsc", "petsc_msplit_ksp.c")).read()
    for kind in ("GMRES", "LSQR"):
        body = re.search(r"static PetscErrorCode KSPSolve_MSplit%s\(KSP ksp\)\n\{(.*?)\n\}" % kind, src, re.S)
        assert body and "MSplitSolveInOrder" in body.group(1), kind
    order = re.search(r"static PetscErrorCode MSplitSolveInOrder\(.*?\n\}", src, re.S).group(0)
    assert order.index("msp_ctx_get_reduction") < order.index("ierr = body(ksp)") < order.rindex("msp_ctx_set_reduction")
    assert src.count("MSPCall(msp_ctx_set_reduction") == order.count("MSPCall(msp_ctx_set_reduction") == 2
    assert src.count("reduction = -1") == 2          # unset: the KSP follows the context's (global) order


@pytest.mark.parametrize("n", [1, 2, 5, 12])
def test_bench_spmv_check_restates_matmult_seqaij(oracle, n):
    """bench.py's spmv_512_csr line checks its last product row by row against poisson3d_rows_product (numpy):
    that restatement is bit for bit the oracle's MatMult_SeqAIJ on the reference's 3D assembly."""
    import numpy as np
    sys.path.insert(0, ROOT)
    import bench
    A = oracle.poisson3d_rows(n, n, n, 0, n)
    x = np.random.default_rng(n).uniform(-1, 1, n ** 3)
    x[0] = -0.0
    yb = np.concatenate([bench.poisson3d_rows_product(x, n, z) for z in range(n)])
    assert np.array_equal(A.mult(x).view(np.uint64), yb.view(np.uint64))


def test_bench_smsm_record_checks():
    """bench.py's SMSM verifications (check_smsm_block for the N = 1 lines, check_configs2_run for an N = 2 run):
    a step that matches the committed record is verified, one changed bit in any checked field is not, and another
    problem has no record."""
    import copy
    import json
    import types
    sys.path.insert(0, ROOT)
    import bench
    blk_rec = json.load(open(bench.SMSM_BLOCK_GOLDEN))["dbr"]
    step = types.SimpleNamespace(lsqr_rnorm=[float.fromhex(h) for h in blk_rec["hist_hex"][:2]],
                                 lsqr_its=list(blk_rec["lsqr_its"][:2]),
                                 inner_its=[v for o in blk_rec["inner_its"][:2] for v in o])
    assert bench.check_smsm_block(step, None, blk_rec, 2) == (True, [])
    bad = copy.deepcopy(step)
    bad.lsqr_rnorm[1] = float.fromhex(blk_rec["hist_hex"][1]) * (1 + 2 ** -52)
    assert bench.check_smsm_block(bad, None, blk_rec, 2) == (False, ["hist_hex"])
    bad = copy.deepcopy(step)
    bad.inner_its[-1] += 1
    assert bench.check_smsm_block(bad, None, blk_rec, 2) == (False, ["inner_its"])
    assert bench.check_smsm_block(step, None, blk_rec, 9)[0] is None      # more steps than the record holds
    assert bench.check_smsm_block(step, None, None, 1)[0] is None

    args = types.SimpleNamespace(smsm_mesh=512, smsm_planes=256, s=20, inner_max_it=20, outer_max_it=70, restart=30,
                                 peclet=None)
    rec = json.load(open(bench.C2_GOLDEN))["cubes"]["512"]
    for rank in (0, 1):
        st = types.SimpleNamespace(lsqr_rnorm=[float.fromhex(h) for h in rec["hist_hex"][:3]],
                                   lsqr_its=list(rec["lsqr_its"][:3]),
                                   inner_its=[rec["inner_its"][o][j][rank] for o in range(3) for j in range(20)])
        assert bench.check_configs2_run(args, st, rank) == (True, [], 3)
        st.lsqr_its[0] -= 1
        assert bench.check_configs2_run(args, st, rank) == (False, ["lsqr_its"], 3)
    other = types.SimpleNamespace(**{**vars(args), "smsm_mesh": 256})
    assert bench.check_configs2_run(other, st, 0)[0] is None


def test_gpu_steps_runner_stops_after_trouble(tmp_path):
    """tools/gpu_steps.sh (the one runner of every GPU session): each step's output in its own log, its exit code
    in status; a failing test run (exit 1) lets the session go on, anything above 1 (a fault, an abort, a time
    limit) ends it there, and a step that outlives its limit is killed (124)."""
    import subprocess
    out = tmp_path / "s"
    r = subprocess.run(["bash", os.path.join(ROOT, "tools", "gpu_steps.sh"), str(out), "a|5|echo hello",
                        "b|5|exit 1", "c|1|sleep 30", "d|5|echo never"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0
    status = (out / "status").read_text().split("\n")
    codes = {ln.split()[0]: ln.split()[1] for ln in status if len(ln.split()) == 3 and ln.split()[1] != "start"}
    assert codes == {"a": "0", "b": "1", "c": "124"}, status
    assert any(ln.startswith("stopping after c (124)") for ln in status)
    assert (out / "a.log").read_text() == "hello\n" and not (out / "d.log").exists()
