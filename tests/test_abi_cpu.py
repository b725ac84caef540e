"""The C-ABI library loads and exports every declared symbol; host-side
helpers agree with the oracle.  No device calls (CPU only)."""
import json
from pathlib import Path

import numpy as np
import pytest

from quicfuscate_amd import _lib as L

GOLDEN = json.loads((Path(__file__).parent / "golden" / "golden.json").read_text())


def test_library_exports_every_header_symbol():
    lib = L._lib()
    syms = L.header_symbols()
    assert len(syms) >= 30
    missing = [s for s in syms if not hasattr(lib, s)]
    assert missing == []
    assert lib.qf_abi_version() == 1


def test_split_table_selftest():
    # all 65,536 products through the v_perm split tables (host emulation)
    assert L._lib().qf_selftest_split_tables() == 0


def test_host_gf_helpers_match_oracle(qf, oracle):
    t = oracle.mul_table_full()
    for a in range(0, 256, 3):
        for b in range(256):
            assert qf.gf_mul(a, b) == t[a, b]
    assert qf.gf_mul_add(3, 7, 0x55) == oracle.mul(3, 7) ^ 0x55
    for a in range(1, 256):
        assert qf.gf_inv(a) == oracle.inv(a)
    with pytest.raises(qf.QfError) as e:
        qf.gf_inv(0)
    assert e.value.status == L.QF_ERANGE


@pytest.mark.parametrize("k,r", [(4, 2), (16, 16), (64, 16), (196, 59), (1, 1), (255, 1)])
def test_cauchy_matches_oracle(qf, oracle, k, r):
    assert qf.cauchy_coefficients(k, r) == oracle.cauchy(k, r).tobytes()


@pytest.mark.parametrize("k,r", [(256, 16), (260, 4), (1024, 8), (197, 60)])
def test_cauchy_erange_where_reference_panics(qf, k, r):
    with pytest.raises(qf.QfError) as e:
        qf.cauchy_coefficients(k, r)
    assert e.value.status == L.QF_ERANGE


def test_framing_roundtrip_and_errors(qf):
    p = qf.Packet(9, bytearray(b"payload-bytes"), 13, False, bytes(range(64)), 64)
    raw = p.to_raw()
    assert raw[0] == 0 and raw[1:3] == (64).to_bytes(2, "big") and raw[3:67] == bytes(range(64))
    q = qf.Packet.from_raw(9, raw)
    assert q.payload() == b"payload-bytes" and q.coefficients == bytes(range(64)) and not q.is_systematic
    s = qf.Packet(1, bytearray(b"abc"), 3, True)
    assert s.to_raw() == b"\x01abc"
    assert qf.Packet.from_raw(1, b"\x01abc").payload() == b"abc"
    for bad in (b"", b"\x00\x01", b"\x00\x00\x05ab"):
        with pytest.raises(qf.QfError):
            qf.Packet.from_raw(0, bad)


def test_option_enum_matches_binding():
    """QF_OPT_* of include/qf_fec.h, in enum order, are the Python binding's
    OPTIONS (the index is the ABI value qf_ctx_set_option takes)."""
    import re

    from quicfuscate_amd import _lib as L

    txt = L.HEADER.read_text()
    enum = txt[txt.index("QF_OPT_FFT_KERNELS = 0"): txt.index("QF_OPT_COUNT")]
    names = [n.lower() for n in re.findall(r"QF_OPT_([A-Z0-9_]+)", enum)]
    assert names == list(L.OPTIONS) and L.QF_OPT_COUNT == len(names)


def test_mirror_rejects_undersized_buffers():
    """fec.encode_batch / decode_batch check every buffer against the shape
    before the library sees a pointer (rec_index: min(k, r) entries per
    generation, include/qf_fec.h)."""
    import pytest
    import torch

    from quicfuscate_amd import fec

    k, r, L, G = 64, 16, 1200, 3
    src = torch.zeros(G * k * L, dtype=torch.uint8)
    with pytest.raises(ValueError, match="rep"):
        fec.encode_batch(src, torch.zeros(G * r * L - 1, dtype=torch.uint8), k, r, L, src_row_stride=L,
                         src_gen_stride=k * L, rep_row_stride=L, rep_gen_stride=r * L, G=G)
    with pytest.raises(ValueError, match="src"):
        fec.encode_batch(src[:-1], torch.zeros(G * r * L, dtype=torch.uint8), k, r, L, src_row_stride=L,
                         src_gen_stride=k * L, rep_row_stride=L, rep_gen_stride=r * L, G=G)
    n = k
    rows = torch.zeros(G * n * L, dtype=torch.uint8)
    idx = torch.zeros(G * n, dtype=torch.int16)
    rec = torch.zeros(G * r * L, dtype=torch.uint8)
    i32 = torch.zeros(G, dtype=torch.int32)
    with pytest.raises(ValueError, match="rec_index"):
        fec.decode_batch(rows, idx, rec, torch.zeros(G * 13, dtype=torch.int16), i32, i32, k, r, L, max_rows=n,
                         row_stride=L, rows_gen_stride=n * L, rec_row_stride=L, rec_gen_stride=r * L, G=G)
    with pytest.raises(ValueError, match="status"):
        fec.decode_batch(rows, idx, rec, torch.zeros(G * r, dtype=torch.int16), i32, i32[:1], k, r, L,
                         max_rows=n, row_stride=L, rows_gen_stride=n * L, rec_row_stride=L,
                         rec_gen_stride=r * L, G=G)


def test_last_error_names_the_failing_hip_call():
    """qf_last_error: a QF_EDEVICE carries the failing HIP call's file:line and
    error name.  Here (no GPU, or an out-of-range
    device ordinal on a GPU host) qf_ctx_create fails in the library."""
    import ctypes
    from quicfuscate_amd import _lib as L

    lib = L._lib()
    h = ctypes.c_void_p()
    s = lib.qf_ctx_create(1 << 20, None, ctypes.byref(h))
    assert s == L.QF_EDEVICE
    why = lib.qf_last_error().decode()
    assert why.startswith("qf_api.hip:") and "hipError" in why, why
    err = L.QfError(s, "ctx")
    assert why in str(err) and err.detail == why
