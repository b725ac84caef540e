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

# Objects still alive when the interpreter exits are not freed through the
# library: the process is ending, and the HIP runtime may already be torn
# down by then (a late hipFree / hipEventSynchronize can crash the exit).
_SHUTDOWN = False


def _mark_shutdown() -> None:
    global _SHUTDOWN
    _SHUTDOWN = True


import atexit as _atexit  # noqa: E402

_atexit.register(_mark_shutdown)

__all__ = [
    "QfError", "Context", "default_context", "init_gf_tables", "gf_mul", "gf_mul_table",
    "gf_mul_add", "gf_inv", "gf_mul_slice", "cauchy_coefficients", "MemoryPool", "Packet",
    "Encoder", "Decoder", "encode_batch", "decode_batch",
    "gf16_mul", "gf16_inv", "cauchy16_coefficients", "encode16_batch", "decode16_batch", "Encoder16", "Decoder16",
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
QF_STREAM_NULL = 1   # qf_fec.h: the device's null stream


class Context:
    """A qf_ctx bound to a device and a HIP stream (default: torch's current)."""

    def __init__(self, device: Optional[int] = None, stream: Optional[int] = None):
        import torch

        if not torch.cuda.is_available():
            raise QfError(L.QF_EDEVICE, "no HIP device visible")
        self.device = torch.cuda.current_device() if device is None else int(device)
        if stream is None:
            stream = torch.cuda.current_stream(self.device).cuda_stream
        if not stream:
            # torch's default stream is the null stream: QF_STREAM_NULL binds
            # the library to it, so its work is ordered with torch's (a NULL
            # stream makes qf_ctx_create allocate its own non-blocking stream,
            # which a torch fill / randint on the default stream does not wait for)
            stream = QF_STREAM_NULL
        h = ctypes.c_void_p()
        check(L._lib().qf_ctx_create(self.device, ctypes.c_void_p(stream), ctypes.byref(h)), "ctx")
        self.handle = h

    def set_stream(self, stream: int) -> None:
        check(L._lib().qf_ctx_set_stream(self.handle, ctypes.c_void_p(stream)))

    def set_option(self, name: str, value: int) -> None:
        """qf_ctx_set_option: a kernel-path option of this context
        (L.OPTIONS: "fft_kernels", "decode_path", ...; include/qf_fec.h)."""
        check(L._lib().qf_ctx_set_option(self.handle, L.OPTIONS[name], int(value)), f"option {name}")

    def option(self, name: str) -> int:
        v = ctypes.c_int64()
        check(L._lib().qf_ctx_get_option(self.handle, L.OPTIONS[name], ctypes.byref(v)), f"option {name}")
        return v.value

    def options(self) -> dict:
        return {n: self.option(n) for n in L.OPTIONS}

    def set_payload_wait(self, event) -> None:
        """qf_ctx_set_payload_wait: the next decode_batch runs its acceptance
        pass at once and its payload pass after `event` (a torch.cuda.Event
        that has been recorded, or a raw hipEvent_t handle; None clears)."""
        h = event if (event is None or isinstance(event, int)) else event.cuda_event
        check(L._lib().qf_ctx_set_payload_wait(self.handle, ctypes.c_void_p(h)), "payload_wait")

    def set_payload_stream(self, stream) -> None:
        """qf_ctx_set_payload_stream: the next decode_batch keeps its
        acceptance pass on this context's stream and runs its payload pass on
        `stream` (a torch.cuda.Stream or a raw hipStream_t; torch's default
        stream maps to the null stream; None clears)."""
        if stream is None:
            h = None
        else:
            h = stream if isinstance(stream, int) else stream.cuda_stream
            h = h or QF_STREAM_NULL
        check(L._lib().qf_ctx_set_payload_stream(self.handle, ctypes.c_void_p(h)), "payload_stream")

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
        if _SHUTDOWN:
            return
        try:
            self.close()
        except Exception:
            pass


_DEFAULT: Optional[Context] = None


_DEFAULT_OPTS: dict = {}


def default_context() -> Context:
    global _DEFAULT, _DEFAULT_OPTS
    if _DEFAULT is None:
        _DEFAULT = Context()
        _DEFAULT_OPTS = _DEFAULT.options()
    return _DEFAULT


def set_default_options(**opts) -> None:
    """Kernel-path options (QF_OPT_*) on the default context, e.g.
    set_default_options(encode_small=0, decode_path=1)."""
    ctx = default_context()
    for n, v in opts.items():
        ctx.set_option(n, v)


def reset_default_options() -> None:
    """The default context's options back to those it was created with."""
    if _DEFAULT is not None and _DEFAULT.handle:
        for n, v in _DEFAULT_OPTS.items():
            _DEFAULT.set_option(n, v)


def _ptr(t) -> int:
    return int(t.data_ptr())


def _need(t, nbytes: int, what: str) -> None:
    """A buffer the library will read or write must hold nbytes (the C ABI
    takes bare pointers: an undersized tensor would be overrun on the device)."""
    if t is None or nbytes <= 0 or not hasattr(t, "numel"):
        return
    have = int(t.numel()) * int(t.element_size())
    if have < nbytes:
        raise ValueError(f"{what}: {have} bytes, the call needs {nbytes}")


def _span(G: int, gen_stride: int, rows: int, row_stride: int, L: int) -> int:
    """Bytes from the first byte of generation 0 to the end of the last row."""
    return 0 if G == 0 or rows == 0 else (G - 1) * gen_stride + (rows - 1) * row_stride + L


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
                 coeff: Optional[bytes] = None, ctx: Optional[Context] = None,
                 zero_tail: bool = False) -> None:
    """qf_encode_batch: repairs of G generations (decoder.rs:172-275).
    zero_tail: QF_ENCODE_ZERO_TAIL (the library may zero [L, round_up(L, 128))
    of each repair row)."""
    _need(src, _span(G, src_gen_stride, k, src_row_stride, Lb), "src")
    _need(rep, _span(G, rep_gen_stride, r, rep_row_stride, Lb), "rep")
    ctx = ctx or default_context()
    sh = L.EncodeShape(k, r, Lb, 1 if zero_tail else 0, src_row_stride, src_gen_stride, rep_row_stride,
                       rep_gen_stride)
    cbuf = None
    if coeff is not None:
        if len(coeff) != k * r:
            raise ValueError("coeff must be r*k bytes")
        cbuf = (ctypes.c_uint8 * len(coeff)).from_buffer_copy(coeff)
    check(L._lib().qf_encode_batch(ctx.handle, ctypes.byref(sh), G, _ptr(src), _ptr(rep),
                                    ctypes.cast(cbuf, ctypes.c_void_p) if cbuf is not None else None),
          "encode_batch")


def pack_gen_descs(descs):
    """A ctypes qf_gen_desc array from dicts / tuples: build it once and pass it
    to encode_batch_desc on every call (a per-call rebuild of thousands of
    descriptors costs milliseconds of host time)."""
    arr = (L.GenDesc * max(1, len(descs)))()
    for i, d in enumerate(descs):
        arr[i] = L.GenDesc(**d) if isinstance(d, dict) else L.GenDesc(*d)
    arr.qf_n = len(descs)
    return arr


def pack_dec_descs(descs):
    """A ctypes qf_dec_desc array (see pack_gen_descs)."""
    arr = (L.DecDesc * max(1, len(descs)))()
    for i, d in enumerate(descs):
        arr[i] = L.DecDesc(**d) if isinstance(d, dict) else L.DecDesc(*d)
    arr.qf_n = len(descs)
    return arr


def encode_batch_desc(src, rep, descs, ctx: Optional[Context] = None) -> None:
    """qf_encode_batch_desc: one call over generations of different (k, r, L)
    at arbitrary offsets.  descs: sequence of dicts or tuples
    (k, r, L, flags, src_offset, src_row_stride, rep_offset, rep_row_stride)."""
    ctx = ctx or default_context()
    arr = descs if isinstance(descs, ctypes.Array) else pack_gen_descs(descs)
    check(L._lib().qf_encode_batch_desc(ctx.handle, arr, getattr(arr, "qf_n", len(arr)), _ptr(src), _ptr(rep)), "encode_batch_desc")


def decode_batch_desc(rows, row_index, rec, rec_index, n_rec, status, descs, ctx: Optional[Context] = None) -> None:
    """qf_decode_batch_desc: descs are dicts / tuples of qf_dec_desc (k, r, L,
    n_rows, rows_offset, row_stride, row_index_offset, rec_offset,
    rec_row_stride, rec_index_offset); n_rec / status: one entry per descriptor."""
    ctx = ctx or default_context()
    arr = descs if isinstance(descs, ctypes.Array) else pack_dec_descs(descs)
    check(L._lib().qf_decode_batch_desc(ctx.handle, arr, getattr(arr, "qf_n", len(arr)), _ptr(rows), _ptr(row_index),
                                         _ptr(rec) if rec is not None else None,
                                         _ptr(rec_index) if rec_index is not None else None, _ptr(n_rec),
                                         _ptr(status)), "decode_batch_desc")


def encode_batch_host(src, rep, k: int, r: int, Lb: int, *, src_row_stride: int, rep_row_stride: int, G: int,
                      coeff: Optional[bytes] = None, ctx: Optional[Context] = None) -> None:
    """qf_encode_batch_host: encode_batch with src / rep in host memory (torch
    CPU tensors, pinned recommended; dense generations); synchronous.  The
    send side of core.rs:252-317, starting from UDP datagrams in host memory."""
    ctx = ctx or default_context()
    sh = L.EncodeShape(k, r, Lb, 0, src_row_stride, k * src_row_stride, rep_row_stride, r * rep_row_stride)
    cbuf = None
    if coeff is not None:
        if len(coeff) != k * r:
            raise ValueError("coeff must be r*k bytes")
        cbuf = (ctypes.c_uint8 * len(coeff)).from_buffer_copy(coeff)
    check(L._lib().qf_encode_batch_host(ctx.handle, ctypes.byref(sh), G, _ptr(src), _ptr(rep),
                                         ctypes.cast(cbuf, ctypes.c_void_p) if cbuf is not None else None),
          "encode_batch_host")


def decode_batch_host(rows, row_index, rec, rec_index, n_rec, status, k: int, r: int, Lb: int, *,
                      max_rows: int, row_stride: int, rows_gen_stride: int, rec_row_stride: int,
                      rec_gen_stride: int, G: int, n_rows=None, row_coeffs=None,
                      ctx: Optional[Context] = None) -> None:
    """qf_decode_batch_host: decode_batch with every buffer in host memory
    (torch CPU tensors, pinned recommended); synchronous."""
    ctx = ctx or default_context()
    sh = L.DecodeShape(k, r, Lb, max_rows, row_stride, rows_gen_stride, rec_row_stride, rec_gen_stride)
    check(L._lib().qf_decode_batch_host(
        ctx.handle, ctypes.byref(sh), G, _ptr(rows), _ptr(row_index),
        _ptr(n_rows) if n_rows is not None else None,
        _ptr(row_coeffs) if row_coeffs is not None else None,
        _ptr(rec) if rec is not None else None, _ptr(rec_index) if rec_index is not None else None,
        _ptr(n_rec), _ptr(status)), "decode_batch_host")


def decode_batch(rows, row_index, rec, rec_index, n_rec, status, k: int, r: int, Lb: int, *,
                 max_rows: int, row_stride: int, rows_gen_stride: int, rec_row_stride: int,
                 rec_gen_stride: int, G: int, n_rows=None, row_coeffs=None,
                 ctx: Optional[Context] = None) -> None:
    """qf_decode_batch: recover erased rows of G generations (decoder.rs:658-791)."""
    em = min(k, r)
    _need(rows, _span(G, rows_gen_stride, max_rows, row_stride, Lb), "rows")
    _need(row_index, 2 * G * max_rows, "row_index")
    _need(rec_index, 2 * G * em, "rec_index (min(k, r) entries per generation)")
    _need(n_rec, 4 * G, "n_rec")
    _need(status, 4 * G, "status")
    if n_rows is not None:
        _need(n_rows, 4 * G, "n_rows")
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
            if len(payload) > pool.block_size:   # "Buffer from pool is too small" (encoder.rs:52-56)
                raise QfError(L.QF_ETOOSMALL, "from_raw: pool buffer too small")
            block = pool.alloc()
            block[: len(payload)] = payload
            payload = block
        return Packet(pid, payload, plen.value, bool(sys_.value), coeffs, clen.value)

    @staticmethod
    def from_block(pid: int, block: bytearray, length: int) -> "Packet":
        """encoder.rs:72-121: parse a received frame held in a pool block of
        `length` valid bytes; the payload is moved to the front of the same
        block (qf_packet_from_block)."""
        lib = L._lib()
        buf = (ctypes.c_uint8 * max(1, len(block))).from_buffer(block) if len(block) else (ctypes.c_uint8 * 1)()
        sys_ = ctypes.c_int(0)
        coeffs = (ctypes.c_uint8 * max(1, len(block)))()
        clen, plen = ctypes.c_uint32(0), ctypes.c_uint32(0)
        check(lib.qf_packet_from_block(buf, len(block), length, ctypes.byref(sys_), coeffs, len(block),
                                       ctypes.byref(clen), ctypes.byref(plen)), "from_block")
        co = bytes(coeffs)[: clen.value] if not sys_.value else None
        return Packet(pid, block, plen.value, bool(sys_.value), co, clen.value)


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
        if _SHUTDOWN:
            return
        try:
            L._lib().qf_encoder_free(self.handle)
        except Exception:
            pass


class Decoder:
    """decoder.rs:658-791 Decoder (first k rows win, systematic id % k).
    k <= 256 decodes by Gauss-Jordan / the Cauchy kernels, k > 256 by the
    Wiedemann strategy (decoder.rs:660-664, 794-975), as Decoder::new picks."""

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

    @property
    def strategy(self) -> str:
        """decoder.rs:520-524 DecodingStrategy chosen by Decoder::new."""
        s = check(L._lib().qf_decoder_strategy(self.handle))
        return "Wiedemann" if s == 1 else "GaussianElimination"

    @property
    def solve_attempts(self) -> int:
        """Projections the last Wiedemann solve tried (1..8; 9 = exact
        elimination decided; 0: none yet / k <= 256)."""
        return check(L._lib().qf_decoder_solve_attempts(self.handle))

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
        if _SHUTDOWN:
            return
        try:
            L._lib().qf_decoder_free(self.handle)
        except Exception:
            pass


# ---------------------------------------------------------------------------
# GF(2^16) Extreme mode (gf_tables.rs:331-380, decoder.rs:10-88, 536-656)
# ---------------------------------------------------------------------------
def gf16_mul(a: int, b: int) -> int:
    """gf_tables.rs:333 gf16_mul with the reduction it intends."""
    return int(L._lib().qf_gf16_mul(a & 0xFFFF, b & 0xFFFF))


def gf16_inv(a: int) -> int:
    """gf_tables.rs:370 gf16_inv; raises for 0."""
    out = ctypes.c_uint16(0)
    check(L._lib().qf_gf16_inv(a & 0xFFFF, ctypes.byref(out)), "gf16_inv")
    return int(out.value)


def cauchy16_coefficients(k: int, r: int) -> list[list[int]]:
    """decoder.rs:77-80 for repairs 0..r-1."""
    buf = (ctypes.c_uint16 * max(1, k * r))()
    check(L._lib().qf_cauchy16_coeffs(k, r, buf), "cauchy16")
    return [list(buf[j * k: (j + 1) * k]) for j in range(r)]


def encode16_batch(src, rep, k: int, r: int, Lb: int, *, src_row_stride: int, src_gen_stride: int,
                   rep_row_stride: int, rep_gen_stride: int, G: int, coeff=None,
                   ctx: Optional[Context] = None) -> None:
    """qf_encode16_batch: GF(2^16) repairs of G generations (Encoder16,
    decoder.rs:33-75).  coeff: optional r x k u16 rows (default Cauchy)."""
    ctx = ctx or default_context()
    sh = L.EncodeShape(k, r, Lb, 0, src_row_stride, src_gen_stride, rep_row_stride, rep_gen_stride)
    cbuf = None
    if coeff is not None:
        flat = [int(v) for row in coeff for v in row]
        if len(flat) != k * r:
            raise ValueError("coeff must be r x k")
        cbuf = (ctypes.c_uint16 * len(flat))(*flat)
    check(L._lib().qf_encode16_batch(ctx.handle, ctypes.byref(sh), G, _ptr(src), _ptr(rep),
                                      ctypes.cast(cbuf, ctypes.c_void_p) if cbuf is not None else None),
          "encode16_batch")


def decode16_batch(rows, row_index, rec, rec_index, n_rec, status, k: int, r: int, Lb: int, *,
                   max_rows: int, row_stride: int, rows_gen_stride: int, rec_row_stride: int,
                   rec_gen_stride: int, G: int, n_rows=None, row_coeffs=None,
                   ctx: Optional[Context] = None) -> None:
    """qf_decode16_batch: Decoder16 (decoder.rs:563-656) over G generations;
    row_coeffs: optional u16 tensor [G, max_rows, k]."""
    ctx = ctx or default_context()
    sh = L.DecodeShape(k, r, Lb, max_rows, row_stride, rows_gen_stride, rec_row_stride, rec_gen_stride)
    check(L._lib().qf_decode16_batch(
        ctx.handle, ctypes.byref(sh), G, _ptr(rows), _ptr(row_index),
        _ptr(n_rows) if n_rows is not None else None,
        _ptr(row_coeffs) if row_coeffs is not None else None,
        _ptr(rec) if rec is not None else None, _ptr(rec_index) if rec_index is not None else None,
        _ptr(n_rec), _ptr(status)), "decode16_batch")


class Encoder16:
    """decoder.rs:10-88 Encoder16 over qf_encoder16_*: sliding window of k
    packets; repair j carries the Cauchy row y = k + j as a big-endian u16
    coefficient block of 2k bytes."""

    def __init__(self, k: int, n: int, max_len: int = 4096, ctx: Optional[Context] = None):
        self.k, self.n, self.max_len = k, n, max_len
        self.ctx = ctx or default_context()
        h = ctypes.c_void_p()
        check(L._lib().qf_encoder16_new(self.ctx.handle, k, n, max_len, ctypes.byref(h)), "Encoder16::new")
        self.handle = h

    def add_source_packet(self, packet: Packet) -> None:
        data = packet.payload()
        buf = (ctypes.c_uint8 * max(1, len(data))).from_buffer_copy(data.ljust(max(1, len(data)), b"\0"))
        check(L._lib().qf_encoder16_add_source_packet(self.handle, packet.id, buf, len(data)), "add_source_packet")

    def generate_repair_packet(self, repair_packet_index: int, pool: Optional[MemoryPool] = None) -> Optional[Packet]:
        out = (ctypes.c_uint8 * self.max_len)()
        coeffs = (ctypes.c_uint8 * (2 * self.k))()
        n = ctypes.c_uint32(0)
        pid = ctypes.c_uint64(0)
        s = L._lib().qf_encoder16_generate_repair_packet(self.handle, repair_packet_index, out, self.max_len,
                                                         ctypes.byref(n), coeffs, ctypes.byref(pid))
        if s == L.QF_ENOTREADY:
            return None
        check(s, "generate_repair_packet")
        block = pool.alloc() if pool is not None else bytearray(max(n.value, 1))
        block[: n.value] = bytes(out)[: n.value]
        return Packet(pid.value, block, n.value, False, bytes(coeffs), 2 * self.k)

    def generate_repairs(self, first: int, count: int) -> list[Packet]:
        stride = (self.max_len + 15) // 16 * 16
        out = (ctypes.c_uint8 * (stride * count))()
        coeffs = (ctypes.c_uint8 * (2 * self.k * count))()
        lens = (ctypes.c_uint32 * count)()
        ids = (ctypes.c_uint64 * count)()
        s = L._lib().qf_encoder16_generate_repairs(self.handle, first, count, out, stride, lens, coeffs, ids)
        if s == L.QF_ENOTREADY:
            return []
        check(s, "generate_repairs")
        raw, cb, kb = bytes(out), bytes(coeffs), 2 * self.k
        return [Packet(ids[q], bytearray(raw[q * stride: q * stride + lens[q]]), lens[q], False,
                       cb[q * kb: (q + 1) * kb], kb) for q in range(count)]

    def __del__(self):  # pragma: no cover
        if _SHUTDOWN:
            return
        try:
            L._lib().qf_encoder16_free(self.handle)
        except Exception:
            pass


class Decoder16:
    """decoder.rs:536-656 Decoder16 over qf_decoder16_*: the first k packets
    (systematic column id % k, repair rows from their big-endian u16
    coefficient blocks), no duplicate filtering.  Systematic payloads are
    carried (F4-style fix) and decoding runs once k rows are present, whatever
    the last row's kind; get_decoded_packets returns the whole generation."""

    def __init__(self, k: int, pool: Optional[MemoryPool] = None, max_len: int = 4096,
                 ctx: Optional[Context] = None):
        self.k = k
        self.ctx = ctx or default_context()
        self.max_len = pool.block_size if pool is not None else max_len
        h = ctypes.c_void_p()
        check(L._lib().qf_decoder16_new(self.ctx.handle, k, self.max_len, ctypes.byref(h)), "Decoder16::new")
        self.handle = h

    @property
    def is_decoded(self) -> bool:
        return bool(check(L._lib().qf_decoder16_is_decoded(self.handle)))

    def add_packet(self, packet: Packet) -> bool:
        data = packet.payload()
        buf = (ctypes.c_uint8 * max(1, len(data))).from_buffer_copy(data.ljust(max(1, len(data)), b"\0"))
        co = None
        if packet.coefficients is not None:
            cb = bytes(packet.coefficients[: packet.coeff_len])
            co = (ctypes.c_uint8 * max(1, len(cb))).from_buffer_copy(cb.ljust(max(1, len(cb)), b"\0"))
        elif not packet.is_systematic:
            raise QfError(L.QF_EINVAL, "missing coeffs")
        s = L._lib().qf_decoder16_add_packet(self.handle, packet.id, 1 if packet.is_systematic else 0, buf,
                                             len(data), ctypes.cast(co, ctypes.c_void_p) if co is not None else None,
                                             packet.coeff_len)
        return bool(check(s, "add_packet"))

    def get_decoded_packets(self) -> list[Packet]:
        stride = (self.max_len + 15) // 16 * 16
        out = (ctypes.c_uint8 * (stride * self.k))()
        lens = (ctypes.c_uint32 * self.k)()
        ids = (ctypes.c_uint64 * self.k)()
        cnt = ctypes.c_uint32(0)
        check(L._lib().qf_decoder16_get_decoded_packets(self.handle, out, stride, lens, ids, ctypes.byref(cnt)),
              "get_decoded_packets")
        raw = bytes(out)
        return [Packet(ids[i], bytearray(raw[i * stride: i * stride + lens[i]]), lens[i], True)
                for i in range(cnt.value)]

    def __del__(self):  # pragma: no cover
        if _SHUTDOWN:
            return
        try:
            L._lib().qf_decoder16_free(self.handle)
        except Exception:
            pass


# ---------------------------------------------------------------------------
# Adaptive FEC driver (adaptive.rs:11-631) over qf_adaptive_*
# ---------------------------------------------------------------------------
import enum
from collections import deque as _deque
from dataclasses import dataclass as _dataclass, field as _field


class FecMode(enum.IntEnum):
    """adaptive.rs:13-21 (with FromStr aliases, 23-37)."""
    Zero = 0
    Light = 1
    Normal = 2
    Medium = 3
    Strong = 4
    Extreme = 5

    @classmethod
    def parse(cls, s: str) -> "FecMode":
        names = {"0": 0, "zero": 0, "1": 1, "light": 1, "leicht": 1, "2": 2, "normal": 2,
                 "3": 3, "medium": 3, "mittel": 3, "4": 4, "strong": 4, "stark": 4, "5": 5, "extreme": 5}
        try:
            return cls(names[s.lower()])
        except KeyError:
            raise ValueError(f"unknown FEC mode {s!r}") from None


def default_windows() -> dict:
    """FecConfig::default_windows (adaptive.rs:352-362)."""
    return {FecMode.Zero: 0, FecMode.Light: 16, FecMode.Normal: 64, FecMode.Medium: 128,
            FecMode.Strong: 512, FecMode.Extreme: 1024}


@_dataclass
class PidConfig:
    kp: float = 1.2
    ki: float = 0.5
    kd: float = 0.1


@_dataclass
class FecConfig:
    """adaptive.rs:338-349, defaults 435-452."""
    lambda_: float = 0.1
    burst_window: int = 20
    hysteresis: float = 0.02
    pid: PidConfig = _field(default_factory=PidConfig)
    initial_mode: FecMode = FecMode.Zero
    kalman_enabled: bool = False
    kalman_q: float = 0.001
    kalman_r: float = 0.01
    window_sizes: dict = _field(default_factory=default_windows)
    max_len: int = 1500

    def to_c(self) -> "L.FecConfig":
        c = L.FecConfig()
        c.lambda_, c.burst_window, c.hysteresis = self.lambda_, self.burst_window, self.hysteresis
        c.kp, c.ki, c.kd = self.pid.kp, self.pid.ki, self.pid.kd
        c.initial_mode = int(self.initial_mode)
        c.kalman_enabled = 1 if self.kalman_enabled else 0
        c.kalman_q, c.kalman_r = self.kalman_q, self.kalman_r
        for m in FecMode:
            c.window_sizes[int(m)] = int(self.window_sizes.get(m, default_windows()[m]))
        c.max_len = self.max_len
        return c

    def validate(self) -> None:
        """FecConfig::validate (adaptive.rs:455-471)."""
        c = self.to_c()
        check(L._lib().qf_fec_config_validate(ctypes.byref(c)), "FecConfig.validate")


class ModeManager:
    """The static parts of adaptive.rs:102-153."""
    CROSS_FADE_LEN = 32
    ALPHA_K = 0.5

    @staticmethod
    def params_for(mode: FecMode, window: int) -> tuple[int, int]:
        k, n = ctypes.c_uint32(), ctypes.c_uint32()
        check(L._lib().qf_mode_params_for(int(mode), window, ctypes.byref(k), ctypes.byref(n)))
        return k.value, n.value

    @staticmethod
    def window_range(mode: FecMode) -> tuple[int, int]:
        lo, hi = ctypes.c_uint32(), ctypes.c_uint32()
        check(L._lib().qf_mode_window_range(int(mode), ctypes.byref(lo), ctypes.byref(hi)))
        return lo.value, hi.value

    @staticmethod
    def overhead_ratio(mode: FecMode) -> float:
        return L._lib().qf_mode_overhead_ratio(int(mode))


class AdaptiveFec:
    """adaptive.rs:326-631.  `ctx=None` with `codec=False` runs the controller
    alone (no GPU); `now` arguments inject the monotonic clock in seconds."""

    def __init__(self, config: FecConfig, pool: Optional[MemoryPool] = None, *, ctx: Optional[Context] = None,
                 codec: bool = True, now: Optional[float] = None):
        self._lib = L._lib()
        self.config = config
        self.pool = pool
        self.ctx = (ctx or default_context()) if codec else None
        h = ctypes.c_void_p()
        c = config.to_c()
        cptr = self.ctx.handle if self.ctx is not None else None
        if now is None:
            check(self._lib.qf_adaptive_new(cptr, ctypes.byref(c), ctypes.byref(h)), "AdaptiveFec.new")
        else:
            check(self._lib.qf_adaptive_new_at(cptr, ctypes.byref(c), float(now), ctypes.byref(h)),
                  "AdaptiveFec.new")
        self.handle = h

    def state(self) -> dict:
        mode, window, k, n = ctypes.c_int32(), ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        tr, left, est = ctypes.c_int32(), ctypes.c_uint32(), ctypes.c_float()
        check(self._lib.qf_adaptive_state(self.handle, ctypes.byref(mode), ctypes.byref(window), ctypes.byref(k),
                                          ctypes.byref(n), ctypes.byref(tr), ctypes.byref(left), ctypes.byref(est)))
        return {"mode": FecMode(mode.value), "window": window.value, "k": k.value, "n": n.value,
                "transitioning": bool(tr.value), "transition_left": left.value, "estimated_loss": est.value}

    def current_mode(self) -> FecMode:
        return self.state()["mode"]

    def is_transitioning(self) -> bool:
        return self.state()["transitioning"]

    def report_loss(self, lost: int, total: int, now: Optional[float] = None) -> None:
        if now is None:
            check(self._lib.qf_adaptive_report_loss(self.handle, lost, total), "report_loss")
        else:
            check(self._lib.qf_adaptive_report_loss_at(self.handle, lost, total, float(now)), "report_loss")

    def on_send(self, pkt: Packet, outgoing_queue) -> int:
        """Pushes the systematic packet and its repairs onto outgoing_queue.
        Returns the status (QF_ERANGE when the field has no code for the
        configuration -- GF(2^8) with k + r > 256, where the reference panics)."""
        cap = self._lib.qf_adaptive_max_send_packets(self.handle)
        stride = max(self.config.max_len, 1)
        st = self.state()
        kmax = max(256, 2 * st["k"])  # coefficient bytes: k (GF(2^8)) or 2k (GF(2^16), Extreme)
        key = (cap, stride, kmax)
        if getattr(self, "_send_bufs", (None,))[0] != key:   # reused across calls
            self._send_bufs = (key, (ctypes.c_uint8 * (cap * stride))(), (ctypes.c_uint8 * (cap * kmax))(),
                               (L.PacketDesc * cap)())
        _, data, co, desc = self._send_bufs
        n = ctypes.c_uint32()
        pay = pkt.payload()
        buf = (ctypes.c_uint8 * max(1, len(pay))).from_buffer_copy(pay.ljust(max(1, len(pay)), b"\0"))
        s = self._lib.qf_adaptive_on_send(self.handle, pkt.id, buf, len(pay), data, stride, co, kmax, desc, cap,
                                          ctypes.byref(n))
        if s not in (L.QF_OK, L.QF_ERANGE):
            check(s, "on_send")
        mv_d, mv_c = memoryview(data), memoryview(co)
        for i in range(n.value):
            d = desc[i]
            payload = bytearray(mv_d[i * stride: i * stride + d.len])
            coeffs = bytes(mv_c[i * kmax: i * kmax + d.coeff_len]) if not d.is_systematic else None
            outgoing_queue.append(Packet(d.id, payload, d.len, bool(d.is_systematic), coeffs, d.coeff_len))
        return s

    def on_receive(self, pkt: Packet) -> list:
        st = self.state()
        cap = max(1, st["k"] + 1024)
        stride = max(self.config.max_len, 1)
        key = (cap, stride)
        if getattr(self, "_recv_bufs", (None,))[0] != key:   # reused across calls
            self._recv_bufs = (key, (ctypes.c_uint8 * (cap * stride))(), (L.PacketDesc * cap)())
        _, data, desc = self._recv_bufs
        n = ctypes.c_uint32()
        pay = pkt.payload()
        buf = (ctypes.c_uint8 * max(1, len(pay))).from_buffer_copy(pay.ljust(max(1, len(pay)), b"\0"))
        co = None
        if pkt.coefficients is not None:
            co = (ctypes.c_uint8 * max(1, pkt.coeff_len)).from_buffer_copy(
                bytes(pkt.coefficients[: pkt.coeff_len]).ljust(max(1, pkt.coeff_len), b"\0"))
        s = self._lib.qf_adaptive_on_receive(self.handle, pkt.id, 1 if pkt.is_systematic else 0, buf, len(pay),
                                             ctypes.cast(co, ctypes.c_void_p) if co is not None else None,
                                             pkt.coeff_len, data, stride, desc, cap, ctypes.byref(n))
        if s == L.QF_EINVAL and not pkt.is_systematic and pkt.coefficients is None:
            raise QfError(s, "Repair packet missing coefficients.")
        check(s, "on_receive")
        mv = memoryview(data)
        return [Packet(desc[i].id, bytearray(mv[i * stride: i * stride + desc[i].len]), desc[i].len, True)
                for i in range(n.value)]

    def close(self) -> None:
        if getattr(self, "handle", None):
            self._lib.qf_adaptive_free(self.handle)
            self.handle = None

    def __del__(self):  # pragma: no cover
        if _SHUTDOWN:
            return
        try:
            self.close()
        except Exception:
            pass


def on_send_batch(fecs, packets, queues=None):
    """AdaptiveFec.on_send for many connections in one call
    (qf_adaptive_on_send_batch): fecs[m] sends packets[m] (a connection may
    appear more than once; its packets are taken in order).  Appends each
    connection's outgoing packets to queues[m] (new lists when None) and
    returns (queues, statuses) -- the same packets and statuses as calling
    fecs[m].on_send(packets[m], queues[m]) for m in order."""
    M = len(fecs)
    if len(packets) != M:
        raise ValueError("one packet per connection")
    queues = [[] for _ in range(M)] if queues is None else queues
    if M == 0:
        return queues, []
    lib = L._lib()
    cap = sum(lib.qf_adaptive_max_send_packets(f.handle) for f in fecs)
    stride = max(max(f.config.max_len for f in fecs), 1)
    kmax = max(256, max(2 * f.state()["k"] for f in fecs))
    conns = (ctypes.c_void_p * M)(*[f.handle for f in fecs])
    ids = (ctypes.c_uint64 * M)(*[p.id for p in packets])
    pays = [p.payload() for p in packets]
    bufs = [(ctypes.c_uint8 * max(1, len(b))).from_buffer_copy(b.ljust(max(1, len(b)), b"\0")) for b in pays]
    data = (ctypes.c_void_p * M)(*[ctypes.addressof(b) for b in bufs])
    lens = (ctypes.c_uint32 * M)(*[len(b) for b in pays])
    out = (ctypes.c_uint8 * (cap * stride))()
    co = (ctypes.c_uint8 * (cap * kmax))()
    desc = (L.PacketDesc * cap)()
    n_out = (ctypes.c_uint32 * M)()
    st = (ctypes.c_int32 * M)()
    check(lib.qf_adaptive_on_send_batch(conns, M, ids, data, lens, out, stride, co, kmax, desc, cap, n_out, st),
          "on_send_batch")
    mv_d, mv_c = memoryview(out), memoryview(co)
    pos = 0
    for m in range(M):
        for i in range(pos, pos + n_out[m]):
            d = desc[i]
            payload = bytearray(mv_d[i * stride: i * stride + d.len])
            coeffs = bytes(mv_c[i * kmax: i * kmax + d.coeff_len]) if not d.is_systematic else None
            queues[m].append(Packet(d.id, payload, d.len, bool(d.is_systematic), coeffs, d.coeff_len))
        pos += n_out[m]
    return queues, list(st)


def on_receive_batch(fecs, packets):
    """AdaptiveFec.on_receive for many connections in one call
    (qf_adaptive_on_receive_batch): fecs[m] receives packets[m].  Returns
    (recovered, statuses): recovered[m] is the list on_receive would return
    (empty on a per-packet error, whose status is in statuses[m])."""
    M = len(fecs)
    if len(packets) != M:
        raise ValueError("one packet per connection")
    if M == 0:
        return [], []
    lib = L._lib()
    cap = max(1, sum(f.state()["k"] + 1024 for f in fecs))
    stride = max(max(f.config.max_len for f in fecs), 1)
    conns = (ctypes.c_void_p * M)(*[f.handle for f in fecs])
    ids = (ctypes.c_uint64 * M)(*[p.id for p in packets])
    sysf = (ctypes.c_int32 * M)(*[1 if p.is_systematic else 0 for p in packets])
    pays = [p.payload() for p in packets]
    bufs = [(ctypes.c_uint8 * max(1, len(b))).from_buffer_copy(b.ljust(max(1, len(b)), b"\0")) for b in pays]
    data = (ctypes.c_void_p * M)(*[ctypes.addressof(b) for b in bufs])
    lens = (ctypes.c_uint32 * M)(*[len(b) for b in pays])
    cbufs = [None if p.coefficients is None else (ctypes.c_uint8 * max(1, p.coeff_len)).from_buffer_copy(
        bytes(p.coefficients[: p.coeff_len]).ljust(max(1, p.coeff_len), b"\0")) for p in packets]
    co = (ctypes.c_void_p * M)(*[None if c is None else ctypes.addressof(c) for c in cbufs])
    cl = (ctypes.c_uint32 * M)(*[p.coeff_len if p.coefficients is not None else 0 for p in packets])
    out = (ctypes.c_uint8 * (cap * stride))()
    desc = (L.PacketDesc * cap)()
    n_out = (ctypes.c_uint32 * M)()
    st = (ctypes.c_int32 * M)()
    check(lib.qf_adaptive_on_receive_batch(conns, M, ids, sysf, data, lens, co, cl, out, stride, desc, cap, n_out,
                                           st), "on_receive_batch")
    mv = memoryview(out)
    res, pos = [], 0
    for m in range(M):
        res.append([Packet(desc[i].id, bytearray(mv[i * stride: i * stride + desc[i].len]), desc[i].len, True)
                    for i in range(pos, pos + n_out[m])])
        pos += n_out[m]
    return res, list(st)
