"""Packet framing (encoder.rs:18-152) on the host.

1. The oracle's framing restatement (oracle/qf_oracle_wire.c) is pinned by
   hand-spelled frames: the reference's frame layout (encoder.rs:17), a k=64
   repair frame of the C2 shape (1 + 2 + 64 + 1200 = 1,267 B), and every
   error branch of from_raw / from_block / to_raw.
2. The library's host framing (qf_packet_to_raw / qf_packet_from_raw /
   qf_packet_from_block) equals the oracle on random frames, including
   malformed ones.  No GPU needed.
"""
import numpy as np
import pytest

from quicfuscate_amd import _lib as L


def _cauchy_row(k, j):
    from quicfuscate_amd import bs_codegen as b

    return bytes(b.cauchy(k, j + 1)[j])


def test_oracle_to_raw_pinned_frames(oracle):
    # systematic: 0x01 | payload, no coefficient header
    s, f = oracle.packet_to_raw(True, b"abc")
    assert s == 0 and f == b"\x01abc"
    # a C2 repair frame: 0x00 | BE u16 k | C[j][0..k) | payload
    k, Lb = 64, 1200
    payload = bytes((7 * t + 3) & 255 for t in range(Lb))
    c = _cauchy_row(k, 5)
    s, f = oracle.packet_to_raw(False, payload, c)
    assert s == 0 and len(f) == 1267
    assert f[:3] == b"\x00\x00\x40" and f[3:67] == c and f[67:] == payload
    # is_systematic and the coefficient Option are independent fields (encoder.rs:134-144)
    s, f = oracle.packet_to_raw(True, b"xy", b"\x05")
    assert f == b"\x01\x00\x01\x05xy"
    s, f = oracle.packet_to_raw(False, b"xy")
    assert f == b"\x00xy"
    # BufferTooShort (encoder.rs:129-131), and the exact fit
    assert oracle.packet_to_raw(False, payload, c, buffer_len=1266)[0] == oracle.FR_BUFFER_TOO_SHORT
    assert oracle.packet_to_raw(False, payload, c, buffer_len=1267)[0] == 0
    # data None: the payload bytes are counted but left as they were (encoder.rs:146-149)
    s, f = oracle.packet_to_raw(True, b"\x00" * 4, None, has_data=False, fill=0xEE)
    assert f == b"\x01" + b"\xee" * 4
    # coeff_len `as u16` truncation (encoder.rs:138)
    s, f = oracle.packet_to_raw(False, b"", bytes(65537), buffer_len=65541)
    assert s == 0 and f[1:3] == b"\x00\x01" and len(f) == 1 + 2 + 65537


def test_oracle_from_raw_pinned(oracle):
    k, Lb = 64, 1200
    c = _cauchy_row(k, 0)
    payload = bytes(range(256)) * 4 + bytes(176)
    frame = b"\x00\x00\x40" + c + payload
    s, sys_, co, pay = oracle.packet_from_raw(frame)
    assert s == 0 and sys_ is False and co == c and pay == payload
    assert oracle.packet_from_raw(b"\x01" + payload)[1:] == (True, None, payload)
    # any first byte other than 1 is a repair frame (encoder.rs:28)
    assert oracle.packet_from_raw(b"\x02\x00\x01\x09zz")[1:] == (False, b"\x09", b"zz")
    assert oracle.packet_from_raw(b"")[0] == oracle.FR_EMPTY
    assert oracle.packet_from_raw(b"\x00\x01")[0] == oracle.FR_NO_COEFF_LEN
    assert oracle.packet_from_raw(b"\x00\x00\x05ab")[0] == oracle.FR_COEFF_TRUNCATED
    assert oracle.packet_from_raw(b"\x00\x00\x00")[1:] == (False, b"", b"")
    assert oracle.packet_from_raw(b"\x01" + bytes(4096))[0] == 0
    assert oracle.packet_from_raw(b"\x01" + bytes(4097))[0] == oracle.FR_POOL_TOO_SMALL
    assert oracle.packet_from_raw(b"\x00\x10\x01" + bytes(4097))[0] == oracle.FR_PANIC


def test_oracle_from_block_pinned(oracle):
    blk = bytearray(b"\x00\x00\x02\xaa\xbbPAYLOAD" + b"\x11" * 7)
    s, sys_, co, plen, out = oracle.packet_from_block(bytes(blk), 12)
    assert s == 0 and sys_ is False and co == b"\xaa\xbb" and plen == 7
    # copy_within(5..12, 0): payload at the front, the rest of the block unchanged
    assert out[:7] == b"PAYLOAD" and out[7:12] == b"AYLOAD"[1:] and out[12:] == b"\x11" * 7
    s, sys_, co, plen, out = oracle.packet_from_block(b"\x01hello\x00\x00", 6)
    assert (s, sys_, co, plen, out[:5]) == (0, True, None, 5, b"hello")
    assert oracle.packet_from_block(b"\x01abc", 0)[0] == oracle.FR_INVALID_LEN
    assert oracle.packet_from_block(b"\x01abc", 5)[0] == oracle.FR_INVALID_LEN
    assert oracle.packet_from_block(b"\x00\x00\x00\x00", 2)[0] == oracle.FR_NO_COEFF_LEN
    assert oracle.packet_from_block(b"\x00\x00\x05abcd", 7)[0] == oracle.FR_COEFF_TRUNCATED


def _qf_code(oracle_status):
    """The library's status for each reference error (include/qf_fec.h)."""
    from tests import oracle_py as o

    return {0: 0, o.FR_EMPTY: L.QF_EINVAL, o.FR_INVALID_LEN: L.QF_EINVAL, o.FR_NO_COEFF_LEN: L.QF_ETOOSMALL,
            o.FR_COEFF_TRUNCATED: L.QF_ETOOSMALL, o.FR_BUFFER_TOO_SHORT: L.QF_ETOOSMALL,
            o.FR_POOL_TOO_SMALL: L.QF_ETOOSMALL, o.FR_PANIC: L.QF_ETOOSMALL}[oracle_status]


def _random_frame(rng):
    kind = rng.integers(0, 6)
    pay = rng.integers(0, 256, int(rng.integers(0, 300)), dtype=np.uint8).tobytes()
    if kind == 0:
        return b"\x01" + pay
    cl = int(rng.integers(0, 80))
    co = rng.integers(0, 256, cl, dtype=np.uint8).tobytes()
    f = bytes([int(rng.choice([0, 2, 0xFF]))]) + cl.to_bytes(2, "big") + co + pay
    if kind == 1:   # truncated somewhere
        f = f[: int(rng.integers(0, len(f) + 1))]
    return f


def test_library_from_raw_equals_oracle(qf, oracle):
    rng = np.random.default_rng(123)
    for _ in range(400):
        f = _random_frame(rng)
        s, sys_, co, pay = oracle.packet_from_raw(f)
        if s:
            with pytest.raises(qf.QfError) as e:
                qf.Packet.from_raw(0, f)
            assert e.value.status == _qf_code(s), f
            continue
        p = qf.Packet.from_raw(7, f)
        assert p.is_systematic == sys_ and p.payload() == pay and p.len == len(pay)
        assert (p.coefficients if not sys_ else None) == co


def test_library_to_raw_equals_oracle(qf, oracle):
    rng = np.random.default_rng(5)
    for _ in range(200):
        sys_ = bool(rng.integers(0, 2))
        pay = rng.integers(0, 256, int(rng.integers(0, 200)), dtype=np.uint8).tobytes()
        co = None if rng.integers(0, 2) else rng.integers(0, 256, int(rng.integers(0, 70)), dtype=np.uint8).tobytes()
        s, want = oracle.packet_to_raw(sys_, pay, co)
        assert s == 0
        got = qf.Packet(1, bytearray(pay), len(pay), sys_, co, len(co) if co is not None else 0).to_raw()
        assert got == want


def test_library_from_block_equals_oracle(qf, oracle):
    rng = np.random.default_rng(9)
    for _ in range(300):
        f = _random_frame(rng)
        block_len = max(len(f), 1) + int(rng.integers(0, 16))
        blk = bytearray(f + rng.integers(0, 256, block_len - len(f), dtype=np.uint8).tobytes())
        length = int(rng.integers(0, len(f) + 2))
        s, sys_, co, plen, out = oracle.packet_from_block(bytes(blk), length)
        if s:
            with pytest.raises(qf.QfError) as e:
                qf.Packet.from_block(0, bytearray(blk), length)
            assert e.value.status == _qf_code(s)
            continue
        p = qf.Packet.from_block(3, blk, length)
        assert p.is_systematic == sys_ and p.len == plen and (p.coefficients if not sys_ else None) == co
        assert bytes(p.data) == out     # the whole block, moved in place


def test_from_raw_pool_too_small(qf):
    pool = qf.MemoryPool(4, 64)
    qf.Packet.from_raw(0, b"\x01" + bytes(64), pool)
    with pytest.raises(qf.QfError) as e:
        qf.Packet.from_raw(0, b"\x01" + bytes(65), pool)
    assert e.value.status == L.QF_ETOOSMALL
