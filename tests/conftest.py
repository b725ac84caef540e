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


@pytest.fixture(autouse=True)
def _restore_default_options():
    """Tests pin kernel paths with fec.set_default_options; every test starts
    from the default context's creation-time options."""
    yield
    fec = sys.modules.get("quicfuscate_amd.fec")
    if fec is not None:
        fec.reset_default_options()


@pytest.fixture
def qf_opts(qf):
    """qf_opts(encode_small=0, ...): options of the default context for one test."""
    return qf.set_default_options
