import os
import subprocess
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parent.parent
if str(REPO) not in sys.path:
    sys.path.insert(0, str(REPO))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X / HIP device (runs on the GPU box)")


def _ensure_oracle():
    lib = REPO / "oracle" / "build" / "liboracle.so"
    if not lib.exists():
        subprocess.run(["make", "-C", str(REPO / "oracle")], check=True, capture_output=True)
    return lib


@pytest.fixture(scope="session")
def oracle():
    _ensure_oracle()
    from tests import oracle_py

    return oracle_py


@pytest.fixture(scope="session")
def qf():
    """The product library (fails loudly when it is not built)."""
    from quicfuscate_amd import fec

    return fec


@pytest.fixture(scope="session")
def gpu_ctx(qf):
    import torch

    assert torch.cuda.is_available(), "gpu test on a host without a HIP device"
    return qf.default_context()
