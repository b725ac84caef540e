"""ctypes binding of libqf_fec.so (the C ABI declared in include/qf_fec.h).

The product path has no fallback: if the library is missing this raises.
torch is imported first so that the process holds one HIP runtime (the
library is linked against the runtime bundled with torch).
"""
from __future__ import annotations

import ctypes
import re
from pathlib import Path

PKG = Path(__file__).resolve().parent
LIB_PATH = PKG / "lib" / "libqf_fec.so"
HEADER = PKG.parent / "include" / "qf_fec.h"

QF_OK = 0
QF_EINVAL = -1
QF_ERANGE = -2
QF_ENOTREADY = -3
QF_ERANK = -4
QF_EDEVICE = -5
QF_ENOMEM = -6
QF_ETOOSMALL = -7

_P = ctypes.c_void_p
_U8 = ctypes.c_uint8
_U16 = ctypes.c_uint16
_U32 = ctypes.c_uint32
_U64 = ctypes.c_uint64
_I = ctypes.c_int
_SZ = ctypes.c_size_t


class QfError(RuntimeError):
    """A negative status returned by libqf_fec."""

    def __init__(self, status: int, what: str = ""):
        self.status = status
        msg = _lib().qf_strerror(status).decode() if _LIB is not None else str(status)
        # QF_EDEVICE: the failing HIP call and any refused launch check (qf_last_error)
        self.detail = _lib().qf_last_error().decode() if (_LIB is not None and status == -5) else ""
        if self.detail:
            msg = f"{msg} [{self.detail}]"
        super().__init__(f"{what}: {msg} ({status})" if what else f"{msg} ({status})")


class EncodeShape(ctypes.Structure):
    _fields_ = [
        ("k", _U32), ("r", _U32), ("L", _U32), ("flags", _U32),
        ("src_row_stride", _U64), ("src_gen_stride", _U64),
        ("rep_row_stride", _U64), ("rep_gen_stride", _U64),
    ]


class DecodeShape(ctypes.Structure):
    _fields_ = [
        ("k", _U32), ("r", _U32), ("L", _U32), ("max_rows", _U32),
        ("row_stride", _U64), ("rows_gen_stride", _U64),
        ("rec_row_stride", _U64), ("rec_gen_stride", _U64),
    ]


class GenDesc(ctypes.Structure):
    """qf_gen_desc (heterogeneous encode batch)."""
    _fields_ = [
        ("k", _U32), ("r", _U32), ("L", _U32), ("flags", _U32),
        ("src_offset", _U64), ("src_row_stride", _U64),
        ("rep_offset", _U64), ("rep_row_stride", _U64),
    ]


class DecDesc(ctypes.Structure):
    """qf_dec_desc (heterogeneous decode batch)."""
    _fields_ = [
        ("k", _U32), ("r", _U32), ("L", _U32), ("n_rows", _U32),
        ("rows_offset", _U64), ("row_stride", _U64), ("row_index_offset", _U64),
        ("rec_offset", _U64), ("rec_row_stride", _U64), ("rec_index_offset", _U64),
    ]


class FecConfig(ctypes.Structure):
    _fields_ = [
        ("lambda_", ctypes.c_float), ("burst_window", _U32), ("hysteresis", ctypes.c_float),
        ("kp", ctypes.c_float), ("ki", ctypes.c_float), ("kd", ctypes.c_float),
        ("initial_mode", ctypes.c_int32), ("kalman_enabled", ctypes.c_int32),
        ("kalman_q", ctypes.c_float), ("kalman_r", ctypes.c_float),
        ("window_sizes", _U32 * 6), ("max_len", _U32),
    ]


class PacketDesc(ctypes.Structure):
    _fields_ = [("id", _U64), ("len", _U32), ("coeff_len", _U32), ("is_systematic", ctypes.c_int32),
                ("reserved", _U32)]


_F = ctypes.c_float
_D = ctypes.c_double

_SIGS = {
    "qf_abi_version": (_I, []),
    "qf_strerror": (ctypes.c_char_p, [_I]),
    "qf_last_error": (ctypes.c_char_p, []),
    "qf_gf256_init": (_I, []),
    "qf_gf256_mul": (_U8, [_U8, _U8]),
    "qf_gf256_mul_add": (_U8, [_U8, _U8, _U8]),
    "qf_gf256_inv": (_I, [_U8, _P]),
    "qf_cauchy_coeffs": (_I, [_U32, _U32, _P]),
    "qf_ctx_create": (_I, [_I, _P, ctypes.POINTER(_P)]),
    "qf_ctx_destroy": (_I, [_P]),
    "qf_ctx_set_stream": (_I, [_P, _P]),
    "qf_ctx_stream": (_P, [_P]),
    "qf_ctx_set_payload_wait": (_I, [_P, _P]),
    "qf_ctx_set_payload_stream": (_I, [_P, _P]),
    "qf_sync": (_I, [_P]),
    "qf_ctx_profile": (_I, [_P, _I]),
    "qf_ctx_set_option": (_I, [_P, _I, ctypes.c_int64]),
    "qf_ctx_get_option": (_I, [_P, _I, _P]),
    "qf_ctx_profile_read": (_I, [_P, _U32, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(_U32),
                                 ctypes.POINTER(ctypes.c_double)]),
    "qf_gf256_mul_slice_dev": (_I, [_P, _P, _P, _P, _SZ]),
    "qf_encode_batch": (_I, [_P, ctypes.POINTER(EncodeShape), _U32, _P, _P, _P]),
    "qf_encode_batch_host": (_I, [_P, ctypes.POINTER(EncodeShape), _U32, _P, _P, _P]),
    "qf_encode_batch_desc": (_I, [_P, ctypes.POINTER(GenDesc), _U32, _P, _P]),
    "qf_decode_batch_desc": (_I, [_P, ctypes.POINTER(DecDesc), _U32, _P, _P, _P, _P, _P, _P]),
    "qf_decode_batch": (_I, [_P, ctypes.POINTER(DecodeShape), _U32, _P, _P, _P, _P, _P, _P, _P, _P]),
    "qf_decode_batch_host": (_I, [_P, ctypes.POINTER(DecodeShape), _U32, _P, _P, _P, _P, _P, _P, _P, _P]),
    "qf_encoder_new": (_I, [_P, _U32, _U32, _U32, ctypes.POINTER(_P)]),
    "qf_encoder_free": (_I, [_P]),
    "qf_encoder_add_source_packet": (_I, [_P, _U64, _P, _U32]),
    "qf_encoder_generate_repair_packet": (_I, [_P, _U32, _P, _U32, _P, _P, _P]),
    "qf_encoder_generate_repairs": (_I, [_P, _U32, _U32, _P, _U32, _P, _P, _P]),
    "qf_encoder_window_len": (_I, [_P]),
    "qf_decoder_new": (_I, [_P, _U32, _U32, ctypes.POINTER(_P)]),
    "qf_decoder_free": (_I, [_P]),
    "qf_decoder_add_packet": (_I, [_P, _U64, _I, _P, _U32, _P, _U32]),
    "qf_decoder_is_decoded": (_I, [_P]),
    "qf_decoder_strategy": (_I, [_P]),
    "qf_decoder_get_decoded_packets": (_I, [_P, _P, _U32, _P, _P, _P]),
    "qf_packet_to_raw": (_I, [_I, _P, _U32, _P, _U32, _P, _U32, _P]),
    "qf_packet_from_raw": (_I, [_P, _U32, _P, _P, _P, _P, _P]),
    "qf_packet_from_block": (_I, [_P, _U32, _U32, _P, _P, _U32, _P, _P]),
    "qf_gf16_mul": (ctypes.c_uint16, [ctypes.c_uint16, ctypes.c_uint16]),
    "qf_gf16_inv": (_I, [ctypes.c_uint16, _P]),
    "qf_cauchy16_coeffs": (_I, [_U32, _U32, _P]),
    "qf_encode16_batch": (_I, [_P, ctypes.POINTER(EncodeShape), _U32, _P, _P, _P]),
    "qf_decode16_batch": (_I, [_P, ctypes.POINTER(DecodeShape), _U32, _P, _P, _P, _P, _P, _P, _P, _P]),
    "qf_encoder16_new": (_I, [_P, _U32, _U32, _U32, ctypes.POINTER(_P)]),
    "qf_encoder16_free": (_I, [_P]),
    "qf_encoder16_add_source_packet": (_I, [_P, _U64, _P, _U32]),
    "qf_encoder16_generate_repair_packet": (_I, [_P, _U32, _P, _U32, _P, _P, _P]),
    "qf_encoder16_generate_repairs": (_I, [_P, _U32, _U32, _P, _U32, _P, _P, _P]),
    "qf_encoder16_window_len": (_I, [_P]),
    "qf_decoder16_new": (_I, [_P, _U32, _U32, ctypes.POINTER(_P)]),
    "qf_decoder16_free": (_I, [_P]),
    "qf_decoder16_add_packet": (_I, [_P, _U64, _I, _P, _U32, _P, _U32]),
    "qf_decoder16_is_decoded": (_I, [_P]),
    "qf_decoder16_get_decoded_packets": (_I, [_P, _P, _U32, _P, _P, _P]),
    "qf_fill_splitmix_dev": (_I, [_P, _P, _SZ, _U64, _U64]),
    "qf_selftest_split_tables": (_I, []),
    "qf_frame_batch_dev": (_I, [_P, ctypes.POINTER(EncodeShape), _U32, _P, _P, _P, _U64, _P]),
    "qf_parse_frames_dev": (_I, [_P, _U32, _U32, _U32, _U32, _U32, _P, _U64, _P, _P, _P, _P, _U64, _U64, _P,
                                 _P, _P]),
    "qf_fec_config_default": (None, [ctypes.POINTER(FecConfig)]),
    "qf_fec_config_validate": (_I, [ctypes.POINTER(FecConfig)]),
    "qf_mode_params_for": (_I, [ctypes.c_int32, _U32, _P, _P]),
    "qf_mode_window_range": (_I, [ctypes.c_int32, _P, _P]),
    "qf_mode_overhead_ratio": (_F, [ctypes.c_int32]),
    "qf_adaptive_new": (_I, [_P, ctypes.POINTER(FecConfig), ctypes.POINTER(_P)]),
    "qf_adaptive_new_at": (_I, [_P, ctypes.POINTER(FecConfig), _D, ctypes.POINTER(_P)]),
    "qf_adaptive_free": (_I, [_P]),
    "qf_adaptive_state": (_I, [_P, _P, _P, _P, _P, _P, _P, _P]),
    "qf_adaptive_max_send_packets": (_U32, [_P]),
    "qf_adaptive_max_receive_packets": (_U32, [_P]),
    "qf_decoder_solve_attempts": (_I, [_P]),
    "qf_adaptive_max_coeff_bytes": (_U32, [_P]),
    "qf_adaptive_on_send": (_I, [_P, _U64, _P, _U32, _P, _U32, _P, _U32, _P, _U32, _P]),
    "qf_adaptive_on_send_batch": (_I, [_P, _U32, _P, _P, _P, _P, _U32, _P, _U32, _P, _U32, _P, _P]),
    "qf_adaptive_on_receive_batch": (_I, [_P, _U32, _P, _P, _P, _P, _P, _P, _P, _U32, _P, _U32, _P, _P]),
    "qf_adaptive_on_receive": (_I, [_P, _U64, _I, _P, _U32, _P, _U32, _P, _U32, _P, _U32, _P]),
    "qf_adaptive_report_loss": (_I, [_P, _U32, _U32]),
    "qf_adaptive_report_loss_at": (_I, [_P, _U32, _U32, _D]),
}

_LIB: ctypes.CDLL | None = None


def header_symbols() -> list[str]:
    """Function names declared in include/qf_fec.h."""
    text = HEADER.read_text()
    return sorted(set(re.findall(r"\b(qf_[a-z0-9_]+)\s*\(", text)))


# QF_OPT_* of include/qf_fec.h, by lower-case name without the prefix
OPTIONS = {n: i for i, n in enumerate([
    "fft_kernels", "bitsliced", "encode_small", "encode_ksplit", "encode_v", "encode_pd", "decode_path",
    "decode_ksplit", "decode_synw", "decode_pd", "decode_chunk", "decode_overlap", "combine_bs",
    "combine_bs_min_q", "combine_split", "prepare_grid", "enc_blocks_per_cu", "dec_blocks_per_cu", "send_fused",
    "send_windows_min_tiles", "send_chunks", "send_profile", "copy_threads", "gf16_dyn", "gf16_logify",
    "gf16_logify_min_blocks", "gf16_lds_gj", "gf16_bitsliced", "gf16_fft", "wiedemann_proj", "gf16_fft_bs", "prepare_lanes", "encode_merged",
    "synw_shared", "combine_wide", "combine_xcd", "combine_jump", "combine_pm24", "sliding_kernels"])}
QF_OPT_COUNT = len(OPTIONS)


def _lib() -> ctypes.CDLL:
    global _LIB
    if _LIB is not None:
        return _LIB
    import torch  # noqa: F401  (one HIP runtime per process)

    if not LIB_PATH.exists():
        raise ImportError(
            f"{LIB_PATH} is not built; run `python -m quicfuscate_amd.build_lib` "
            "(there is no CPU fallback for the FEC path)")
    lib = ctypes.CDLL(str(LIB_PATH))
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _LIB = lib
    return lib


def check(status: int, what: str = "") -> int:
    if status < 0:
        raise QfError(status, what)
    return status
