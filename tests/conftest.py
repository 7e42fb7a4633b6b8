import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP library)")


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
