"""Python mirror of QuicFuscate's `quicfuscate::fec` API on the MI355X library.

Names, argument meaning and error behaviour follow the reference
(src/fec/{gf_tables,decoder,encoder}.rs) so that the parity tests read like
the reference's own tests (tests/fec.rs, src/fec/mod.rs).  Every payload
operation runs on the GPU through libqf_fec.so; there is no CPU fallback.

Reference panics become exceptions: gf_inv(0) and Cauchy rows with
k + r > 256 raise QfError(QF_ERANGE).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Optional

from . import _lib as L
from ._lib import QfError, check

__all__ = [
    "QfError", "Context", "default_context", "init_gf_tables", "gf_mul", "gf_mul_table",
    "gf_mul_add", "gf_inv", "gf_mul_slice", "cauchy_coefficients", "MemoryPool", "Packet",
    "Encoder", "Decoder", "encode_batch", "decode_batch",
]


# ---------------------------------------------------------------------------
# GF(2^8) helpers (gf_tables.rs)
# ---------------------------------------------------------------------------
def init_gf_tables() -> None:
    """gf_tables.rs:392 init_gf_tables (idempotent)."""
    check(L._lib().qf_gf256_init())


def gf_mul(a: int, b: int) -> int:
    """gf_tables.rs:283 gf_mul; identical to gf_mul_table for every pair."""
    return int(L._lib().qf_gf256_mul(a & 0xFF, b & 0xFF))


gf_mul_table = gf_mul  # gf_tables.rs:47 (the semantic contract)


def gf_mul_add(a: int, b: int, c: int) -> int:
    """gf_tables.rs:327 gf_mul_add = gf_mul(a, b) ^ c."""
    return int(L._lib().qf_gf256_mul_add(a & 0xFF, b & 0xFF, c & 0xFF))


def gf_inv(a: int) -> int:
    """gf_tables.rs:304 gf_inv; the reference panics for 0, this raises."""
    out = ctypes.c_uint8(0)
    check(L._lib().qf_gf256_inv(a & 0xFF, ctypes.byref(out)), "gf_inv")
    return int(out.value)


def cauchy_coefficients(k: int, r: int) -> bytes:
    """decoder.rs:280-298 for repairs 0..r-1, row-major r x k."""
    buf = (ctypes.c_uint8 * max(1, k * r))()
    check(L._lib().qf_cauchy_coeffs(k, r, buf), "cauchy")
    return bytes(buf)[: k * r]


# ---------------------------------------------------------------------------
# Device context
# ---------------------------------------------------------------------------
class Context:
    """A qf_ctx bound to a device and a HIP stream (default: torch's current)."""

    def __init__(self, device: Optional[int] = None, stream: Optional[int] = None):
        import torch

        if not torch.cuda.is_available():
            raise QfError(L.QF_EDEVICE, "no HIP device visible")
        self.device = torch.cuda.current_device() if device is None else int(device)
        if stream is None:
            stream = torch.cuda.current_stream(self.device).cuda_stream
        h = ctypes.c_void_p()
        check(L._lib().qf_ctx_create(self.device, ctypes.c_void_p(stream), ctypes.byref(h)), "ctx")
        self.handle = h

    def set_stream(self, stream: int) -> None:
        check(L._lib().qf_ctx_set_stream(self.handle, ctypes.c_void_p(stream)))

    def sync(self) -> None:
        check(L._lib().qf_sync(self.handle), "sync")

    def profile(self, on: bool) -> None:
        """Start (clearing totals) or stop per-kernel event timing."""
        check(L._lib().qf_ctx_profile(self.handle, 1 if on else 0), "profile")

    def kernel_times(self) -> dict:
        """{kernel name: (launches, total ms)} accumulated while profiling."""
        out = {}
        i = 0
        lib = L._lib()
        while True:
            name, n, ms = ctypes.c_char_p(), ctypes.c_uint32(), ctypes.c_double()
            s = lib.qf_ctx_profile_read(self.handle, i, ctypes.byref(name), ctypes.byref(n), ctypes.byref(ms))
            if s == L.QF_EINVAL:
                return out
            check(s, "profile_read")
            out[name.value.decode()] = (n.value, ms.value)
            i += 1

    def close(self) -> None:
        if getattr(self, "handle", None):
            L._lib().qf_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass


_DEFAULT: Optional[Context] = None


def default_context() -> Context:
    global _DEFAULT
    if _DEFAULT is None:
        _DEFAULT = Context()
    return _DEFAULT


def _ptr(t) -> int:
    return int(t.data_ptr())


def gf_mul_slice(a: bytes, b: bytes, ctx: Optional[Context] = None) -> bytes:
    """gf_tables.rs:255 gf_mul_slice: element-wise a[i]*b[i], on the device."""
    import torch

    if len(a) != len(b):
        raise ValueError("gf_mul_slice: length mismatch (reference asserts)")
    ctx = ctx or default_context()
    n = len(a)
    if n == 0:
        return b""
    da = torch.frombuffer(bytearray(a), dtype=torch.uint8).to(f"cuda:{ctx.device}")
    db = torch.frombuffer(bytearray(b), dtype=torch.uint8).to(f"cuda:{ctx.device}")
    out = torch.empty_like(da)
    torch.cuda.current_stream(ctx.device).synchronize()
    check(L._lib().qf_gf256_mul_slice_dev(ctx.handle, _ptr(da), _ptr(db), _ptr(out), n), "mul_slice")
    ctx.sync()
    return bytes(out.cpu().numpy().tobytes())


# ---------------------------------------------------------------------------
# Batched device API (torch uint8 tensors on the context's device)
# ---------------------------------------------------------------------------
def encode_batch(src, rep, k: int, r: int, Lb: int, *, src_row_stride: int, src_gen_stride: int,
                 rep_row_stride: int, rep_gen_stride: int, G: int,
                 coeff: Optional[bytes] = None, ctx: Optional[Context] = None) -> None:
    """qf_encode_batch: repairs of G generations (decoder.rs:172-275)."""
    ctx = ctx or default_context()
    sh = L.EncodeShape(k, r, Lb, 0, src_row_stride, src_gen_stride, rep_row_stride, rep_gen_stride)
    cbuf = None
    if coeff is not None:
        if len(coeff) != k * r:
            raise ValueError("coeff must be r*k bytes")
        cbuf = (ctypes.c_uint8 * len(coeff)).from_buffer_copy(coeff)
    check(L._lib().qf_encode_batch(ctx.handle, ctypes.byref(sh), G, _ptr(src), _ptr(rep),
                                    ctypes.cast(cbuf, ctypes.c_void_p) if cbuf is not None else None),
          "encode_batch")


def decode_batch(rows, row_index, rec, rec_index, n_rec, status, k: int, r: int, Lb: int, *,
                 max_rows: int, row_stride: int, rows_gen_stride: int, rec_row_stride: int,
                 rec_gen_stride: int, G: int, n_rows=None, row_coeffs=None,
                 ctx: Optional[Context] = None) -> None:
    """qf_decode_batch: recover erased rows of G generations (decoder.rs:658-791)."""
    ctx = ctx or default_context()
    sh = L.DecodeShape(k, r, Lb, max_rows, row_stride, rows_gen_stride, rec_row_stride, rec_gen_stride)
    check(L._lib().qf_decode_batch(
        ctx.handle, ctypes.byref(sh), G, _ptr(rows), _ptr(row_index),
        _ptr(n_rows) if n_rows is not None else None,
        _ptr(row_coeffs) if row_coeffs is not None else None,
        _ptr(rec) if rec is not None else None, _ptr(rec_index) if rec_index is not None else None,
        _ptr(n_rec), _ptr(status)), "decode_batch")


# ---------------------------------------------------------------------------
# Packet / MemoryPool / Encoder / Decoder (encoder.rs, decoder.rs, optimize.rs)
# ---------------------------------------------------------------------------
class MemoryPool:
    """Stand-in for optimize.rs:417 MemoryPool: hands out zeroed blocks.

    The reference pool is a host allocator; payloads handed to the GPU path
    are copied into HBM by the encoder/decoder, so this only fixes the block
    size (the maximum packet length)."""

    def __init__(self, capacity: int, block_size: int):
        self.capacity = capacity
        self.block_size = block_size

    def alloc(self) -> bytearray:
        return bytearray(self.block_size)


@dataclass
class Packet:
    """encoder.rs:4-12."""
    id: int
    data: Optional[bytearray]
    len: int
    is_systematic: bool
    coefficients: Optional[bytes] = None
    coeff_len: int = 0

    def clone(self) -> "Packet":
        return Packet(self.id, bytearray(self.data) if self.data is not None else None, self.len,
                      self.is_systematic, self.coefficients, self.coeff_len)

    clone_for_encoder = clone  # encoder.rs:156 (deep copy)

    def payload(self) -> bytes:
        return bytes(self.data[: self.len]) if self.data is not None else b""

    def to_raw(self) -> bytes:
        """encoder.rs:124-152."""
        lib = L._lib()
        cap = self.len + 3 + self.coeff_len
        out = (ctypes.c_uint8 * max(1, cap))()
        n = ctypes.c_uint32(0)
        pay = (ctypes.c_uint8 * max(1, self.len)).from_buffer_copy(self.payload().ljust(max(1, self.len), b"\0"))
        co = None
        if self.coefficients is not None:
            co = (ctypes.c_uint8 * max(1, self.coeff_len)).from_buffer_copy(
                bytes(self.coefficients[: self.coeff_len]).ljust(max(1, self.coeff_len), b"\0"))
        check(lib.qf_packet_to_raw(1 if self.is_systematic else 0,
                                   ctypes.cast(co, ctypes.c_void_p) if co is not None else None,
                                   self.coeff_len, pay, self.len, out, cap, ctypes.byref(n)), "to_raw")
        return bytes(out)[: n.value]

    @staticmethod
    def from_raw(pid: int, raw: bytes, pool: Optional[MemoryPool] = None) -> "Packet":
        """encoder.rs:18-68."""
        lib = L._lib()
        buf = (ctypes.c_uint8 * max(1, len(raw))).from_buffer_copy(raw if raw else b"\0")
        sys_ = ctypes.c_int(0)
        cptr, pptr = ctypes.c_void_p(), ctypes.c_void_p()
        clen, plen = ctypes.c_uint32(0), ctypes.c_uint32(0)
        check(lib.qf_packet_from_raw(buf, len(raw), ctypes.byref(sys_), ctypes.byref(cptr),
                                     ctypes.byref(clen), ctypes.byref(pptr), ctypes.byref(plen)),
              "from_raw")
        base = ctypes.addressof(buf)
        coeffs = None
        if cptr.value:
            off = cptr.value - base
            coeffs = bytes(raw[off: off + clen.value])
        off = pptr.value - base
        payload = bytearray(raw[off: off + plen.value])
        if pool is not None:
            block = pool.alloc()
            block[: len(payload)] = payload
            payload = block
        return Packet(pid, payload, plen.value, bool(sys_.value), coeffs, clen.value)


class Encoder:
    """decoder.rs:155-299 Encoder (GF(2^8), Cauchy coefficients)."""

    def __init__(self, k: int, n: int, max_len: int = 4096, ctx: Optional[Context] = None):
        self.k, self.n = k, n
        self.ctx = ctx or default_context()
        h = ctypes.c_void_p()
        check(L._lib().qf_encoder_new(self.ctx.handle, k, n, max_len, ctypes.byref(h)), "Encoder::new")
        self.handle = h
        self.max_len = max_len

    def add_source_packet(self, packet: Packet) -> None:
        data = packet.payload()
        buf = (ctypes.c_uint8 * max(1, len(data))).from_buffer_copy(data.ljust(max(1, len(data)), b"\0"))
        check(L._lib().qf_encoder_add_source_packet(self.handle, packet.id, buf, len(data)),
              "add_source_packet")

    def generate_repair_packet(self, repair_packet_index: int, pool: Optional[MemoryPool] = None) -> Optional[Packet]:
        """Returns None while the window holds fewer than k packets."""
        out = (ctypes.c_uint8 * self.max_len)()
        coeffs = (ctypes.c_uint8 * self.k)()
        n = ctypes.c_uint32(0)
        pid = ctypes.c_uint64(0)
        s = L._lib().qf_encoder_generate_repair_packet(self.handle, repair_packet_index, out, self.max_len,
                                                       ctypes.byref(n), coeffs, ctypes.byref(pid))
        if s == L.QF_ENOTREADY:
            return None
        check(s, "generate_repair_packet")
        block = pool.alloc() if pool is not None else bytearray(max(n.value, 1))
        block[: n.value] = bytes(out)[: n.value]
        return Packet(pid.value, block, n.value, False, bytes(coeffs), self.k)

    def generate_repairs(self, first: int, count: int) -> list[Packet]:
        """All repairs first..first+count-1 of the window in one launch."""
        stride = (self.max_len + 15) // 16 * 16
        out = (ctypes.c_uint8 * (stride * count))()
        coeffs = (ctypes.c_uint8 * (self.k * count))()
        lens = (ctypes.c_uint32 * count)()
        ids = (ctypes.c_uint64 * count)()
        s = L._lib().qf_encoder_generate_repairs(self.handle, first, count, out, stride, lens, coeffs, ids)
        if s == L.QF_ENOTREADY:
            return []
        check(s, "generate_repairs")
        raw = bytes(out)
        cb = bytes(coeffs)
        return [Packet(ids[q], bytearray(raw[q * stride: q * stride + lens[q]]), lens[q], False,
                       cb[q * self.k: (q + 1) * self.k], self.k) for q in range(count)]

    def __del__(self):  # pragma: no cover
        try:
            L._lib().qf_encoder_free(self.handle)
        except Exception:
            pass


class Decoder:
    """decoder.rs:658-791 Decoder (first k rows win, systematic id % k)."""

    def __init__(self, k: int, pool: Optional[MemoryPool] = None, max_len: int = 4096,
                 ctx: Optional[Context] = None):
        self.k = k
        self.ctx = ctx or default_context()
        self.max_len = pool.block_size if pool is not None else max_len
        h = ctypes.c_void_p()
        check(L._lib().qf_decoder_new(self.ctx.handle, k, self.max_len, ctypes.byref(h)), "Decoder::new")
        self.handle = h

    @property
    def is_decoded(self) -> bool:
        return bool(check(L._lib().qf_decoder_is_decoded(self.handle)))

    def add_packet(self, packet: Packet) -> bool:
        """Returns is_decoded; raises for a repair packet without coefficients."""
        data = packet.payload()
        buf = (ctypes.c_uint8 * max(1, len(data))).from_buffer_copy(data.ljust(max(1, len(data)), b"\0"))
        co = None
        if packet.coefficients is not None:
            cb = bytes(packet.coefficients[: packet.coeff_len])
            co = (ctypes.c_uint8 * max(1, len(cb))).from_buffer_copy(cb.ljust(max(1, len(cb)), b"\0"))
        elif not packet.is_systematic:
            raise QfError(L.QF_EINVAL, "Repair packet missing coefficients.")
        s = L._lib().qf_decoder_add_packet(self.handle, packet.id, 1 if packet.is_systematic else 0, buf,
                                           len(data), ctypes.cast(co, ctypes.c_void_p) if co is not None else None,
                                           packet.coeff_len)
        return bool(check(s, "add_packet"))

    def get_decoded_packets(self) -> list[Packet]:
        stride = (self.max_len + 15) // 16 * 16
        out = (ctypes.c_uint8 * (stride * self.k))()
        lens = (ctypes.c_uint32 * self.k)()
        ids = (ctypes.c_uint64 * self.k)()
        cnt = ctypes.c_uint32(0)
        check(L._lib().qf_decoder_get_decoded_packets(self.handle, out, stride, lens, ids, ctypes.byref(cnt)),
              "get_decoded_packets")
        raw = bytes(out)
        res = []
        for i in range(cnt.value):
            block = bytearray(self.max_len)
            block[: lens[i]] = raw[i * stride: i * stride + lens[i]]
            res.append(Packet(ids[i], block, lens[i], True))
        return res

    def __del__(self):  # pragma: no cover
        try:
            L._lib().qf_decoder_free(self.handle)
        except Exception:
            pass
