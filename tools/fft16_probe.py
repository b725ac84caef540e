#!/usr/bin/env python3
"""A few GF(2^16) FFT encodes of 16 Extreme windows (k = r = 1,024, L = 1,200)
for counter passes:  rocprofv3 --pmc ... -- python3 tools/fft16_probe.py"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    import torch

    from quicfuscate_amd import fec as qf

    k, r, L, G = 1024, 1024, 1200, 16
    rs = 1216
    src = torch.randint(0, 256, (G * k * rs,), dtype=torch.uint8, device="cuda")
    rep = torch.empty(G * r * rs, dtype=torch.uint8, device="cuda")
    for _ in range(3):
        qf.encode16_batch(src, rep, k, r, L, src_row_stride=rs, src_gen_stride=k * rs, rep_row_stride=rs,
                          rep_gen_stride=r * rs, G=G)
    qf.default_context().sync()
    print("FFT16_PROBE_OK")


if __name__ == "__main__":
    main()
