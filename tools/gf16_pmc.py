#!/usr/bin/env python3
"""Minimal GF(2^16) encode driver for rocprofv3 --pmc passes: the batched
(k 64, r 16) and Extreme window (k = r = 1,024) encodes, nothing else on the
device besides the input fill.

    rocprofv3 --pmc <counters> -- python3 tools/gf16_pmc.py
"""
from __future__ import annotations

import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))


def main():
    import torch

    from quicfuscate_amd import fec as qf

    ctx = qf.default_context()
    for k, r, L, G in ((64, 16, 1200, 2048), (1024, 1024, 1200, 1), (1024, 1024, 1200, 16)):
        rs = (L + 15) // 16 * 16
        src = torch.randint(0, 256, (G * k * rs,), dtype=torch.uint8, device="cuda")
        rep = torch.empty(G * r * rs, dtype=torch.uint8, device="cuda")
        for _ in range(2):
            qf.encode16_batch(src, rep, k, r, L, src_row_stride=rs, src_gen_stride=k * rs, rep_row_stride=rs,
                              rep_gen_stride=r * rs, G=G)
        ctx.sync()
        print(k, r, G, "ok", flush=True)
        if G == 1:
            # one window's decode: rows assembled on the host (no device gather kernels)
            import numpy as np

            e = 512
            rng = np.random.default_rng(0)
            s_h = src.view(k, rs).cpu().numpy()
            r_h = rep.view(r, rs).cpu().numpy()
            lost = np.sort(rng.choice(k, e, replace=False))
            keep = np.setdiff1d(np.arange(k), lost)
            idx = np.concatenate([keep, k + np.arange(e)]).astype(np.uint16)
            rows = torch.from_numpy(np.concatenate([s_h[keep], r_h[:e]]).reshape(-1).copy()).cuda()
            t_idx = torch.from_numpy(idx.view(np.int16).copy()).cuda()
            rec = torch.empty(e * rs, dtype=torch.uint8, device="cuda")
            ri = torch.empty(e, dtype=torch.int16, device="cuda")
            nrec = torch.empty(1, dtype=torch.int32, device="cuda")
            st = torch.empty(1, dtype=torch.int32, device="cuda")
            for _ in range(2):
                qf.decode16_batch(rows, t_idx, rec, ri, nrec, st, k, r, L, max_rows=k, row_stride=rs,
                                  rows_gen_stride=k * rs, rec_row_stride=rs, rec_gen_stride=e * rs, G=1)
            ctx.sync()
            assert int(st.cpu()[0]) == 0
            got = rec.view(e, rs).cpu().numpy()[:, :L]
            assert (got == s_h[lost][:, :L]).all()
            print("decode ok", flush=True)


if __name__ == "__main__":
    main()
