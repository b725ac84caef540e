"""The bit-sliced GF(2^16) encode schedule (quicfuscate_amd/gf16_codegen.py)
on the CPU: the generated kernels' term lists, run by the numpy model on one
lane's 4 units, equal the oracle's Encoder16 (oracle/qf_oracle16.c,
decoder.rs:10-88 with the intended reduction).  The device kernels
run the same term lists (tests/test_gpu_gf16.py::test_encode16_bitsliced)."""
import numpy as np
import pytest

from quicfuscate_amd import gf16_codegen as g16


def test_transpose_is_involution():
    rng = np.random.default_rng(3)
    x = rng.integers(0, 2**32, 16, dtype=np.uint32)
    assert np.array_equal(g16.transpose16(g16.transpose16(x)), x)
    # plane b holds raw bit b of every half-word: one set bit moves predictably
    for m in range(16):
        for c in (0, 5, 17, 31):
            y = np.zeros(16, np.uint32)
            y[m] = np.uint32(1 << c)
            t = g16.transpose16(y)
            assert [int(v) for v in t].count(0) == 15 and int(t[c % 16]) == 1 << (16 * (c // 16) + m)


def test_field_and_cauchy_rows():
    assert g16.mul(0x8000, 2) == 0x100B           # x^16 = x^12 + x^3 + x + 1 (0x1100B)
    for a in (1, 2, 0x1234, 0xFFFF):
        assert g16.mul(a, g16.inv(a)) == 1
    C = g16.cauchy16(64, 16)
    assert C[0][0] == g16.inv(64) and C[15][63] == g16.inv(63 ^ 79)


@pytest.mark.parametrize("k,r", g16.GF16_BS_CONFIGS)
def test_schedule_matches_oracle(oracle, k, r):
    rng = np.random.default_rng(k * 100 + r)
    rows = rng.integers(0, 256, (k, 64), dtype=np.uint8)
    rows[0, :6] = 0                                # zero symbols
    rows[1, :2] = 255
    out = g16.emulate(k, r, rows)
    ref = oracle.encode16(rows, r)                 # the lane's 64 bytes as one 64-B row set
    assert np.array_equal(out, ref)


def test_generated_source_shape():
    src = g16.generate_all()
    for k, r in g16.GF16_BS_CONFIGS:
        name = g16.kernel_name(k, r)
        assert f"__global__ void __launch_bounds__(256, 2) {name}(" in src
        assert f'{name}, "{name}"' in src
    # every row closes with the accumulator barrier (no reassociation across rows)
    k, r = 16, 4
    one = g16.generate(k, r)
    assert one.count('asm volatile("" :') == k * r      # one per row and repair
