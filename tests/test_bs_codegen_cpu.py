"""The generated bit-sliced Cauchy kernel, executed by the IR emulator on
CPU against the oracle: results, memory bounds and load/wait discipline.
(The same IR is emitted as gfx950 assembly; tests/test_gpu_encode.py runs
the assembled kernel on the device.)"""
import numpy as np
import pytest

from quicfuscate_amd import bs_codegen as bs


@pytest.mark.parametrize("k,r,pd,L,G,waves", [
    (8, 4, 2, 96, 5, 2),     # whole 32-byte chunks
    (8, 4, 2, 80, 7, 3),     # L % 32 == 16: a half chunk per row
    (5, 3, 3, 64, 4, 1),     # odd k, prefetch deeper than k
    (1, 1, 1, 64, 3, 1),
    (16, 16, 4, 1200, 3, 2), # a full-width accumulator set
])
def test_emulated_kernel_matches_oracle(oracle, k, r, pd, L, G, waves):
    spec = bs.KernelSpec(k, r, pd)
    ops = bs.generate(spec)
    rng = np.random.default_rng(k * 100 + r + L)
    srs = L + 16 * (k % 3)          # row stride > L on some shapes
    sgs = k * srs + 32
    drs = L + 32
    dgs = r * drs + 16
    src = rng.integers(0, 256, G * sgs, dtype=np.uint8)
    dst = np.full(G * dgs, 0xEE, np.uint8)
    emu = bs.Emulator(ops)
    SRC, DST = 0x10000000, 0x40000000
    emu.add_buffer(SRC, src)
    emu.add_buffer(DST, dst)
    ka = bs.kernargs(SRC, DST, sgs, dgs, srs, drs, L, G, waves * 4)
    for wg in range(waves):
        for w in range(4):
            emu.run_wave(ka, wg, w)
    for g in range(G):
        rows = np.stack([src[g * sgs + i * srs: g * sgs + i * srs + L] for i in range(k)])
        want = oracle.encode(rows, r)
        for j in range(r):
            off = g * dgs + j * drs
            assert (dst[off: off + L] == want[j]).all(), (g, j)
            assert (dst[off + L: off + drs] == 0xEE).all()


def test_emulator_catches_missing_wait():
    spec = bs.KernelSpec(4, 2, 2)
    ops = [op for op in bs.generate(spec) if not (op.name == "s_waitcnt_vm" and op.args[0] == 2)]
    src = np.zeros(4 * 64 * 2, np.uint8)
    dst = np.zeros(2 * 64 * 2, np.uint8)
    emu = bs.Emulator(ops)
    emu.add_buffer(0x1000, src)
    emu.add_buffer(0x900000, dst)
    with pytest.raises(bs.EmuError):
        emu.run_wave(bs.kernargs(0x1000, 0x900000, 256, 128, 64, 64, 64, 2, 4), 0, 0)


def test_magic_division():
    for U in (2, 3, 5, 37, 38, 64, 100, 282, 1000):
        m, sh = bs.magic_for(U)
        for f in list(range(0, 5000)) + [2**22 + 17, 2**24 - 1, 2**30 + 12345]:
            assert ((f * m) >> 32) >> sh == f // U


def test_mul_matrix_rows_reproduce_field():
    for c in range(256):
        rows = bs.mul_matrix_rows(c)
        for x in (1, 2, 3, 0x53, 0x80, 0xFF):
            y = 0
            for b in range(8):
                y |= (bin(rows[b] & x).count("1") & 1) << b
            assert y == bs.gf_mul(c, x)
