"""bench.py's own checks on the GPU box: the N > 1 line names its transport, --require-rccl refuses a run
that fell back to the host transport, the N = 1 step verifies its result against the committed oracle
record (tests/golden/configs1_seq.json), and the N > 1 line carries the multi-rank check against
tests/golden/smsm_ranks.json."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--variant", "smsm", "--smsm-mesh", "64", "--smsm-planes", "16", "--steps", "1", "--warmup", "0",
         "--no-timing"]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _launch(n, args, timeout=240, rccl_hosts=False):
    """bench.py --gpus n under torch.distributed.run, as the driver launches it.  rccl_hosts: every rank under its
    own NCCL_HOSTID (tests/rccl_rank_env.sh), so RCCL accepts n ranks on this box's one GPU."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={_port()}"]
    if rccl_hosts:
        cmd += ["--no-python", os.path.join(ROOT, "tests", "rccl_rank_env.sh"), sys.executable]
    cmd += [os.path.join(ROOT, "bench.py"), "--gpus", str(n)] + args
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd=ROOT, env=env)


def _json(out):
    return json.loads([ln for ln in out.splitlines() if ln.startswith("{")][-1])


def test_two_rank_rehearsal_reports_host_transport():
    """Two ranks sharing the one GPU over gloo: the library communicator takes its host transport, and the
    bench line says so in config.transport (not only in the workload prose)."""
    r = _launch(2, ["--backend", "gloo"] + SMALL)
    assert r.returncode == 0, r.stderr[-3000:]
    out = _json(r.stdout)
    assert out["n_gpus"] == 2 and out["config"]["transport"] == "host"
    # the post-timing multi-rank check: SMSM-global over the same communicator, bitwise the oracle record
    assert out["verified"] is True and out["verification"]["mismatch"] == [], out.get("verification")
    assert "smsm_ranks.json" in out["verification"]["reference"]


def test_three_rank_rehearsal_is_verified():
    """Three ranks (an interior block with two neighbours): the multi-rank check reproduces the oracle's
    three-block record bit for bit on every rank."""
    r = _launch(3, ["--backend", "gloo"] + SMALL)
    assert r.returncode == 0, r.stderr[-3000:]
    out = _json(r.stdout)
    assert out["n_gpus"] == 3 and out["verified"] is True, out.get("verification")


def test_require_rccl_refuses_host_transport():
    """--require-rccl (the driver's scaling runs): a run whose library communicator is not RCCL exits non-zero
    on every rank before any timing, and prints no bench line."""
    r = _launch(2, ["--backend", "gloo", "--require-rccl"] + SMALL)
    assert r.returncode != 0
    assert "--require-rccl" in r.stderr
    assert not any(ln.startswith("{") for ln in r.stdout.splitlines())


def test_single_gpu_line_is_verified():
    """N = 1: the timed GMRES step (configs[1]) equals the committed DBR oracle record -- iterations, reason, every
    history entry, SHA-256 of x -- and the line says verified: true; the CSR-storage rerun is verified too."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "1", "--warmup", "0",
                        "--no-smsm-n1", "--no-spmv512", "--no-cpu-baseline", "--no-seq-mode", "--no-seq-smsm"],
                       capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    out = _json(r.stdout)
    assert out["verified"] is True and out["verification"]["mismatch"] == []
    assert out["same_run_csr_storage"]["verified"] is True
    assert out["config"]["transport"] == "none"


@pytest.mark.parametrize("n", [2, 3, 8])
def test_rccl_multi_rank_line_is_verified(n):
    """The driver's N > 1 path itself -- torch.distributed.run, the nccl (RCCL) process group, LibComm's library
    RCCL communicator, --require-rccl -- with n ranks on this box's one GPU, each under its own NCCL_HOSTID (RCCL's
    socket transport instead of xGMI: correctness, not speed).  The line says transport rccl, and the post-timing
    SMSM-global check over that communicator reproduces the oracle's n-block record bit for bit on every rank.
    n = 8 is the driver's scaling world size: the first time its exact launch runs is here, not on the 8-GPU node."""
    r = _launch(n, ["--require-rccl"] + SMALL, rccl_hosts=True, timeout=240 if n < 8 else 480)
    assert r.returncode == 0, r.stderr[-3000:]
    out = _json(r.stdout)
    assert out["n_gpus"] == n and out["config"]["transport"] == "rccl"
    assert out["verified"] is True and out["verification"]["mismatch"] == [], out.get("verification")
