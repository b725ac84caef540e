#!/usr/bin/env python3
"""Debug aid: the C5 pass kernels (plain / FFT / merged) at jumbo rows against
the oracle, reporting where each variant's repairs differ."""
import sys
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
from quicfuscate_amd import fec as qf  # noqa: E402
from tests import oracle_py as oracle  # noqa: E402

k, r = int(sys.argv[1]), int(sys.argv[2])
G = int(sys.argv[3]) if len(sys.argv) > 3 else 72
L, RS, drs = 9000, 9008, 9088
ctx = qf.default_context()
gen = torch.Generator(device="cuda").manual_seed(k + r)
src = torch.randint(0, 256, ((G + 1) * k * RS,), dtype=torch.uint8, device="cuda", generator=gen)
s = src.cpu().numpy()
want = {g: oracle.encode(s[g * k * RS:(g + 1) * k * RS].reshape(k, RS)[:, :L], r) for g in (0, 1, G // 2, G - 1)}
outs = {}
for merged in (0, 1):
    for fft in (0, 1):
        qf.set_default_options(encode_merged=merged, fft_kernels=fft)
        rep = torch.full((G * r * drs,), 0xA5, dtype=torch.uint8, device="cuda")
        ctx.profile(True)
        qf.encode_batch(src, rep, k, r, L, src_row_stride=RS, src_gen_stride=k * RS, rep_row_stride=drs,
                        rep_gen_stride=r * drs, G=G, zero_tail=True, ctx=ctx)
        ctx.sync()
        names = list(ctx.kernel_times())
        ctx.profile(False)
        got = rep.view(G, r, drs).cpu().numpy()
        outs[(merged, fft)] = got
        for g, w in want.items():
            bad = [(j, int(np.argmax(got[g, j, :L] != w[j])), int((got[g, j, :L] != w[j]).sum()))
                   for j in range(r) if (got[g, j, :L] != w[j]).any()]
            print(f"merged={merged} fft={fft} g={g} kernels={names} bad={bad[:8]} n={len(bad)}", flush=True)
base = outs[(0, 0)]
for key, got in outs.items():
    d = np.argwhere(got != base)
    print(key, "differs from (0, 0) at", len(d), "bytes; first", d[:5].tolist(),
          "gens", sorted(set(d[:, 0].tolist()))[:20], "rows", sorted(set(d[:, 1].tolist()))[:50], flush=True)
    for g in sorted(set(d[:, 0].tolist()))[:3]:
        w = oracle.encode(s[g * k * RS:(g + 1) * k * RS].reshape(k, RS)[:, :L], r)
        print("  g", g, "base ok", bool((base[g, :, :L] == w).all()), "variant ok", bool((got[g, :, :L] == w).all()))
