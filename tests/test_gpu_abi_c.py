"""The C ABI driven from plain C (tests/abi_c/qf_abi_test.c): batch encode /
decode, heterogeneous batches, the Encoder / Decoder objects, the adaptive
driver's on_send / on_receive / state and the framing calls, each checked
against the CPU oracle -- the caller a reference-side integration would be,
without Python in between."""
import subprocess
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
ABI = Path(__file__).resolve().parent / "abi_c"


def test_c_caller_against_oracle():
    exe = ABI / "build" / "qf_abi_test"
    if not exe.exists():   # normally built by __graft_entry__.build()
        subprocess.run(["make", "-C", str(ABI)], check=True, capture_output=True, timeout=120)
    # the product library here is the /opt/rocm-linked build: the process
    # holds ROCm's HIP runtime and nothing of torch
    ldd = subprocess.run(["ldd", str(exe)], capture_output=True, text=True, timeout=60).stdout
    assert "libqf_fec_rocm.so" in ldd and "torch" not in ldd, ldd
    hip = [l for l in ldd.splitlines() if "libamdhip64" in l]
    assert hip and all("/opt/rocm" in l for l in hip), ldd
    p = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
    assert p.stdout.strip().splitlines()[-1] == "ALL OK"
    for part in ("batch ok", "options ok", "desc ok", "objects ok", "adaptive ok", "adaptive reuse ok", "adaptive batch ok", "framing ok"):
        assert part in p.stdout
