"""ctypes wrapper of oracle/build/liboracle.so -- TEST INFRASTRUCTURE ONLY.

The CPU restatement of src/fec (oracle/qf_oracle.c) used as the parity
checker.  Never imported by the product package.
"""
from __future__ import annotations

import ctypes
from pathlib import Path

import numpy as np

_LIB_PATH = Path(__file__).resolve().parent.parent / "oracle" / "build" / "liboracle.so"
_lib = ctypes.CDLL(str(_LIB_PATH))
_P = ctypes.c_void_p
_U32 = ctypes.c_uint32
_SZ = ctypes.c_size_t
_lib.cpu_encode_table.argtypes = [ctypes.c_uint32] * 4 + [_P, _P, ctypes.c_uint32]
_lib.cpu_encode_avx2.argtypes = [ctypes.c_uint32] * 4 + [_P, _P, ctypes.c_uint32]
_lib.cpu_has_avx2.argtypes = []
_lib.cpu_encode_gfni.argtypes = [ctypes.c_uint32] * 4 + [_P, _P, ctypes.c_uint32]
_lib.cpu_encode_clmul.argtypes = [ctypes.c_uint32] * 4 + [_P, _P, ctypes.c_uint32]
_lib.cpu_encode_clmul_dispatch.argtypes = [ctypes.c_uint32] * 4 + [_P, _P, ctypes.c_uint32]
_lib.cpu_has_gfni.argtypes = []
_lib.cpu_has_pclmul.argtypes = []
_lib.cpu_set_pinning.argtypes = [ctypes.c_int]
_lib.cpu_pinning.argtypes = []
_lib.cpu_gf_mul_loop.argtypes = [ctypes.c_int, ctypes.c_uint64]
_lib.oracle_gf_mul.restype = ctypes.c_uint8
_lib.oracle_gf_mul.argtypes = [ctypes.c_uint8, ctypes.c_uint8]
_lib.oracle_gf_mul_shift.restype = ctypes.c_uint8
_lib.oracle_gf_mul_shift.argtypes = [ctypes.c_uint8, ctypes.c_uint8]
_lib.oracle_gf_mul_clmul_fold.restype = ctypes.c_uint8
_lib.oracle_gf_mul_clmul_fold.argtypes = [ctypes.c_uint8, ctypes.c_uint8]
_lib.oracle_gf_inv.argtypes = [ctypes.c_uint8, _P]
_lib.oracle_gf_tables.argtypes = [_P, _P]
_lib.oracle_gf_mul_slice.argtypes = [_P, _P, _P, _SZ]
_lib.oracle_cauchy_coeffs.argtypes = [_U32, _U32, _P]
_lib.oracle_encode_window.argtypes = [_U32, _U32, _U32, _P, _SZ, _P, _P, _SZ]
_lib.oracle_encode_window_clmul_fold.argtypes = [_U32, _U32, _U32, _P, _SZ, _P, _P, _SZ]
_lib.oracle_decode_generation.argtypes = [_U32, _U32, _U32, _P, _P, _SZ, _P, _P, _SZ, _P]
_lib.oracle_decode_generation_as_written.argtypes = [_U32, _U32, _U32, _P, _P, _SZ, _P, _P, _SZ]
_lib.oracle_wiedemann_decode.argtypes = [_U32, _U32, _U32, _P, _P, _SZ, _P, _P, _SZ, _P, _P]
_lib.oracle_fill_splitmix.argtypes = [_P, _SZ, ctypes.c_uint64, ctypes.c_uint64]
_lib.oracle_gf_init()

OK, ENOTREADY, ERANK, EINVAL, ERANGE = 0, -3, -4, -1, -2


def _p(a: np.ndarray | None):
    return None if a is None else a.ctypes.data


def tables() -> tuple[np.ndarray, np.ndarray]:
    e = np.zeros(512, np.uint8)
    lg = np.zeros(256, np.uint8)
    _lib.oracle_gf_tables(_p(e), _p(lg))
    return e, lg


def mul(a: int, b: int) -> int:
    return int(_lib.oracle_gf_mul(a, b))


def mul_shift(a: int, b: int) -> int:
    return int(_lib.oracle_gf_mul_shift(a, b))


def mul_clmul_fold(a: int, b: int) -> int:
    return int(_lib.oracle_gf_mul_clmul_fold(a, b))


def mul_table_full() -> np.ndarray:
    """256 x 256 product table via oracle_gf_mul_slice."""
    a = np.repeat(np.arange(256, dtype=np.uint8), 256)
    b = np.tile(np.arange(256, dtype=np.uint8), 256)
    out = np.zeros(65536, np.uint8)
    _lib.oracle_gf_mul_slice(_p(a), _p(b), _p(out), 65536)
    return out.reshape(256, 256)


def inv(a: int) -> int | None:
    o = ctypes.c_uint8(0)
    return None if _lib.oracle_gf_inv(a, ctypes.byref(o)) else int(o.value)


def cauchy(k: int, r: int) -> np.ndarray | None:
    out = np.zeros((r, k), np.uint8)
    return None if _lib.oracle_cauchy_coeffs(k, r, _p(out)) else out


def encode(src: np.ndarray, r: int, coeff: np.ndarray | None = None, L: int | None = None) -> np.ndarray:
    """src: (k, stride) uint8 rows -> (r, L) repairs (decoder.rs:172-275)."""
    src = np.ascontiguousarray(src, dtype=np.uint8)
    k, stride = src.shape
    L = stride if L is None else L
    rep = np.zeros((r, max(L, 1)), np.uint8)
    c = None if coeff is None else np.ascontiguousarray(coeff, dtype=np.uint8)
    s = _lib.oracle_encode_window(k, r, L, _p(src), stride, _p(c), _p(rep), rep.shape[1])
    if s != 0:
        raise ValueError(f"oracle encode status {s}")
    return rep[:, :L]


def cpu_encode(kind: str, src: np.ndarray, r: int, threads: int = 1) -> np.ndarray:
    """Comparison encoders of oracle/cpu_variants.c over dense generations:
    src (G, k, L) -> (G, r, L).  kind: "table", "avx2", "gfni", "clmul" (the
    reference's as-written per-byte PCLMULQDQ fold without its dispatch: a
    lower bound) or "clmul_dispatch" (the same, paying optimize.rs:385-408's
    per-byte FeatureDetector + HashMap dispatch).  Both clmul kinds are timing
    only: their output is the defective fold product, SURVEY F3."""
    src = np.ascontiguousarray(src, dtype=np.uint8)
    G, k, L = src.shape
    rep = np.zeros((G, r, L), np.uint8)
    fn = {"table": _lib.cpu_encode_table, "avx2": _lib.cpu_encode_avx2, "gfni": _lib.cpu_encode_gfni,
          "clmul": _lib.cpu_encode_clmul, "clmul_dispatch": _lib.cpu_encode_clmul_dispatch}[kind]
    s = fn(k, r, L, G, _p(src), _p(rep), threads)
    if s != 0:
        raise ValueError(f"cpu_encode({kind}) status {s}")
    return rep


def has_avx2() -> bool:
    return bool(_lib.cpu_has_avx2())


_lib.cpu_decode.argtypes = [ctypes.c_int] + [ctypes.c_uint32] * 4 + [_P, _P, _P, ctypes.c_uint32]


def cpu_decode(kind: str, k: int, row_index: np.ndarray, rows: np.ndarray, threads: int = 1) -> np.ndarray:
    """Host decode of oracle/cpu_variants.c over G generations on `threads`
    threads: row_index (G, n) and rows (G, n, L) in arrival order -> every
    source row (G, k, L).  kind "table" = the oracle's Gauss-Jordan
    (decoder.rs:720-783, table gf_mul); "clmul_dispatch" = the same
    elimination with the reference's per-byte dispatched CLMUL-fold product
    (timing only)."""
    rows = np.ascontiguousarray(rows, dtype=np.uint8)
    ri = np.ascontiguousarray(row_index, dtype=np.uint16)
    G, n, L = rows.shape
    out = np.zeros((G, k, L), np.uint8)
    s = _lib.cpu_decode({"table": 0, "clmul_dispatch": 4}[kind], k, L, G, n, _p(ri), _p(rows), _p(out), threads)
    if s != 0 and kind == "table":
        raise ValueError(f"cpu_decode({kind}) status {s}")
    return out


def has_cpu_kind(kind: str) -> bool:
    """Whether this host can run cpu_encode(kind)."""
    return {"table": lambda: True, "avx2": _lib.cpu_has_avx2, "gfni": _lib.cpu_has_gfni,
            "clmul": _lib.cpu_has_pclmul, "clmul_dispatch": _lib.cpu_has_pclmul}[kind]() != 0


def encode_clmul_fold(src: np.ndarray, r: int) -> np.ndarray:
    src = np.ascontiguousarray(src, dtype=np.uint8)
    k, L = src.shape
    rep = np.zeros((r, L), np.uint8)
    _lib.oracle_encode_window_clmul_fold(k, r, L, _p(src), L, None, _p(rep), L)
    return rep


def decode(k: int, row_index, rows: np.ndarray, row_coeffs: np.ndarray | None = None):
    """rows: (n, L) in arrival order -> (status, out (k, L), received mask)."""
    rows = np.ascontiguousarray(rows, dtype=np.uint8)
    n, L = rows.shape
    ri = np.ascontiguousarray(row_index, dtype=np.uint16)
    out = np.zeros((k, max(L, 1)), np.uint8)
    mask = np.zeros(k, np.uint8)
    rc = None if row_coeffs is None else np.ascontiguousarray(row_coeffs, dtype=np.uint8)
    s = _lib.oracle_decode_generation(k, L, n, _p(ri), _p(rows), L, _p(rc), _p(out), out.shape[1], _p(mask))
    return s, out[:, :L], mask


def wiedemann(k: int, row_index, rows: np.ndarray, row_coeffs: np.ndarray | None = None):
    """decoder.rs:794-975 (fixed, checked; oracle/qf_oracle_wiedemann.c): rows
    (n, L) in arrival order, row_coeffs (n, k) for repair rows -> (status, out
    (k, L), received mask, init vectors tried)."""
    rows = np.ascontiguousarray(rows, dtype=np.uint8)
    n, L = rows.shape
    ri = np.ascontiguousarray(row_index, dtype=np.uint16)
    out = np.zeros((k, max(L, 1)), np.uint8)
    mask = np.zeros(k, np.uint8)
    tries = ctypes.c_uint32(0)
    rc = None if row_coeffs is None else np.ascontiguousarray(row_coeffs, dtype=np.uint8)
    s = _lib.oracle_wiedemann_decode(k, L, n, _p(ri), _p(rows), L, _p(rc), _p(out), out.shape[1], _p(mask),
                                     ctypes.byref(tries))
    return s, out[:, :L], mask, int(tries.value)


def decode_as_written(k: int, row_index, rows: np.ndarray):
    rows = np.ascontiguousarray(rows, dtype=np.uint8)
    n, L = rows.shape
    ri = np.ascontiguousarray(row_index, dtype=np.uint16)
    out = np.zeros((k, L), np.uint8)
    s = _lib.oracle_decode_generation_as_written(k, L, n, _p(ri), _p(rows), L, None, _p(out), L)
    return s, out


def fill_splitmix(n: int, seed: int, word_offset: int = 0) -> np.ndarray:
    out = np.zeros(n, np.uint8)
    _lib.oracle_fill_splitmix(_p(out), n, seed, word_offset)
    return out


# ---- packet framing (oracle/qf_oracle_wire.c, encoder.rs:18-152) -------------
FR_EMPTY, FR_NO_COEFF_LEN, FR_COEFF_TRUNCATED, FR_POOL_TOO_SMALL = -10, -11, -12, -13
FR_INVALID_LEN, FR_BUFFER_TOO_SHORT, FR_PANIC = -14, -15, -16
_SZP = ctypes.POINTER(ctypes.c_size_t)
_lib.oracle_packet_to_raw.argtypes = [ctypes.c_int, ctypes.c_int, _P, _U32, ctypes.c_int, _P, _U32, _P, _SZ, _P]
_lib.oracle_packet_from_raw.argtypes = [_P, _SZ, _SZ, _P, _P, _P, _P, _P]
_lib.oracle_packet_from_block.argtypes = [_P, _SZ, _SZ, _P, _P, _P, _P]


def packet_to_raw(is_systematic: bool, payload: bytes, coeffs: bytes | None = None, buffer_len: int | None = None,
                  has_data: bool = True, fill: int = 0):
    """encoder.rs:124-152 -> (status, frame bytes).  coeffs None = no
    coefficient block (the Option is None)."""
    payload = bytes(payload)
    cb = np.frombuffer(coeffs, np.uint8).copy() if coeffs else np.zeros(1, np.uint8)
    pb = np.frombuffer(payload, np.uint8).copy() if payload else np.zeros(1, np.uint8)
    need = len(payload) + 1 + (2 + len(coeffs) if coeffs is not None else 0)
    n = need if buffer_len is None else buffer_len
    buf = np.full(max(n, 1), fill, np.uint8)
    w = ctypes.c_size_t(0)
    s = _lib.oracle_packet_to_raw(1 if is_systematic else 0, 0 if coeffs is None else 1, _p(cb),
                                  0 if coeffs is None else len(coeffs), 1 if has_data else 0, _p(pb), len(payload),
                                  _p(buf), n, ctypes.byref(w))
    return s, (buf[: w.value].tobytes() if s == 0 else b"")


def packet_from_raw(raw: bytes, block_size: int = 4096):
    """encoder.rs:18-68 -> (status, is_systematic, coeffs, payload)."""
    raw = bytes(raw)
    rb = np.frombuffer(raw, np.uint8).copy() if raw else np.zeros(1, np.uint8)
    sy, cl = ctypes.c_int(0), ctypes.c_uint32(0)
    co, po, ln = ctypes.c_size_t(0), ctypes.c_size_t(0), ctypes.c_size_t(0)
    s = _lib.oracle_packet_from_raw(_p(rb), len(raw), block_size, ctypes.byref(sy), ctypes.byref(cl),
                                    ctypes.byref(co), ctypes.byref(po), ctypes.byref(ln))
    if s:
        return s, None, None, None
    coeffs = raw[co.value: co.value + cl.value] if not sy.value else None
    return s, bool(sy.value), coeffs, raw[po.value: po.value + ln.value]


def packet_from_block(block: bytes, length: int):
    """encoder.rs:72-121 -> (status, is_systematic, coeffs, payload_len, block after the move)."""
    b = np.frombuffer(bytes(block), np.uint8).copy()
    co = np.zeros(len(block) + 1, np.uint8)
    sy, cl, pl = ctypes.c_int(0), ctypes.c_uint32(0), ctypes.c_size_t(0)
    s = _lib.oracle_packet_from_block(_p(b), len(block), length, ctypes.byref(sy), _p(co), ctypes.byref(cl),
                                      ctypes.byref(pl))
    if s:
        return s, None, None, None, None
    return s, bool(sy.value), (co[: cl.value].tobytes() if not sy.value else None), pl.value, b.tobytes()


# ---- GF(2^16) Extreme mode (oracle/qf_oracle16.c) ---------------------------
_lib.oracle_gf16_mul.restype = ctypes.c_uint16
_lib.oracle_gf16_mul.argtypes = [ctypes.c_uint16, ctypes.c_uint16]
_lib.oracle_gf16_inv.argtypes = [ctypes.c_uint16, _P]
_lib.oracle_cauchy16.argtypes = [_U32, _U32, _P]
_lib.oracle_encode16.argtypes = [_U32, _U32, _U32, _P, _SZ, _P, _P, _SZ]
_lib.oracle_decode16.argtypes = [_U32, _U32, _U32, _P, _P, _SZ, _P, _P, _SZ, _P]


def mul16(a: int, b: int) -> int:
    return int(_lib.oracle_gf16_mul(a, b))


def inv16(a: int) -> int | None:
    o = ctypes.c_uint16()
    return None if _lib.oracle_gf16_inv(a, ctypes.byref(o)) else int(o.value)


def cauchy16(k: int, r: int) -> np.ndarray | None:
    out = np.zeros((r, k), np.uint16)
    return None if _lib.oracle_cauchy16(k, r, _p(out)) else out


def encode16(src: np.ndarray, r: int, coeff: np.ndarray | None = None) -> np.ndarray:
    """src: (k, L) uint8 -> (r, L) repairs (big-endian u16 symbols)."""
    src = np.ascontiguousarray(src, dtype=np.uint8)
    k, L = src.shape
    rep = np.zeros((r, L), np.uint8)
    c = None if coeff is None else np.ascontiguousarray(coeff, dtype=np.uint16)
    s = _lib.oracle_encode16(k, r, L, _p(src), L, _p(c), _p(rep), L)
    assert s == 0, s
    return rep


def decode16(k: int, row_index, rows: np.ndarray, row_coeffs: np.ndarray | None = None):
    """rows: (n, L) in arrival order -> (status, out (k, L), received mask)."""
    rows = np.ascontiguousarray(rows, dtype=np.uint8)
    n, L = rows.shape
    ri = np.ascontiguousarray(row_index, dtype=np.uint16)
    out = np.zeros((k, max(L, 1)), np.uint8)
    mask = np.zeros(k, np.uint8)
    rc = None if row_coeffs is None else np.ascontiguousarray(row_coeffs, dtype=np.uint16)
    s = _lib.oracle_decode16(k, L, n, _p(ri), _p(rows), L, _p(rc), _p(out), out.shape[1], _p(mask))
    return s, out[:, :L], mask


GF_MUL_LOOP_KINDS = {"table": 0, "dispatch": 1, "sse2": 2, "avx512": 3, "avx2": 4}
_lib.cpu_clmul_fold_pair.argtypes = [ctypes.c_int, ctypes.c_uint8, ctypes.c_uint8]
_lib.cpu_clmul_fold_pair.restype = ctypes.c_int


def clmul_fold_pair(kind: str, a: int, b: int) -> int:
    """One product of the reference's CLMUL member `kind` (sse2 / avx512 /
    avx2, gf_tables.rs:76-141; the defective fold), -3 if absent."""
    return _lib.cpu_clmul_fold_pair(GF_MUL_LOOP_KINDS[kind], a, b)


def gf_mul_loop(kind: str, iters: int) -> int:
    """oracle/cpu_variants.c cpu_gf_mul_loop: the reference's 1,024-pair
    gf_mul micro-benchmark (benches/gf_bitslice_bench.rs:17-102); returns acc
    or -3 when the host lacks the instructions."""
    return _lib.cpu_gf_mul_loop(GF_MUL_LOOP_KINDS[kind], iters)


def set_pinning(on: bool) -> None:
    """Pin cpu_encode's worker w to the w-th allowed CPU."""
    _lib.cpu_set_pinning(1 if on else 0)
