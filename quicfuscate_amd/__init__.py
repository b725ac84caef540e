"""quicfuscate_amd -- MI355X-native GF(2^8) RLNC FEC path of QuicFuscate.

The hot path (batched Cauchy encode, Gauss-Jordan erasure decode) runs in
hand-written gfx950 HIP kernels behind the C ABI in include/qf_fec.h
(libqf_fec.so).  `quicfuscate_amd.fec` mirrors the reference's Rust API.
"""
from . import _lib  # noqa: F401

__all__ = ["fec"]
