import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP library)")


# The kernel, GMRES, SEQ-order, W-free, DV, KAT, LSQR, Gram and full-size configs suites run first; the suites
# that spawn processes (mpiexec C hosts, multi-process IPC/LibComm runs, the gloo bench rehearsal) and the
# memory-heavy per-GPU AMAM blocks run last, so that under `pytest -x` one host-side failure there can no longer
# hide the device parity record collected before it.
_LATE = ["test_gpu_amam_configs.py", "test_gpu_async_mp.py", "test_gpu_libcomm_mp.py", "test_gpu_bench.py",
         "test_gpu_c_host.py", "test_gpu_c_drivers.py", "test_gpu_nb8.py"]


def pytest_collection_modifyitems(session, config, items):
    def rank(item):
        name = os.path.basename(str(item.fspath))
        return _LATE.index(name) + 1 if name in _LATE else 0
    items[:] = sorted(items, key=rank)   # stable: the order inside each file is kept


@pytest.fixture(scope="session")
def oracle():
    import pyoracle
    pyoracle.build()
    return pyoracle


@pytest.fixture(scope="session")
def ctx():
    import torch  # noqa: F401  -- one HIP runtime shared with torch
    from medane_tchakorom_ufc_thesis_repository_amd.petsc import Context, device_count
    if device_count() == 0:
        pytest.fail("no GPU visible: the gpu tests need an MI355X (no CPU fallback exists)")
    c = Context(0)
    yield c
