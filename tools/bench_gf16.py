#!/usr/bin/env python3
"""GF(2^16) Extreme-mode throughput on the MI355X (diagnostic, not the bench
line): encode16 and decode16 for the batched generation shape (k=64, r=16,
L=1200) and one Extreme window (adaptive.rs:131, k=1024, n=2k), per-kernel
times from the context's HIP events, beside the oracle's single-thread time.

    python tools/bench_gf16.py [--G 8192] [--out gpurun_out/gf16_bench.json]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))


def _r16(x):
    return (x + 15) // 16 * 16


def timed(ctx, fn, reps):
    import torch

    fn()
    ctx.sync()
    ctx.profile(True)
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    ctx.sync()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / reps * 1e3
    kt = {n: (c / reps, ms / reps) for n, (c, ms) in ctx.kernel_times().items()}
    ctx.profile(False)
    return wall, kt


def main():
    import torch

    from quicfuscate_amd import fec as qf
    from tests import oracle_py as oracle

    ap = argparse.ArgumentParser()
    ap.add_argument("--G", type=int, default=8192)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--out", default="gpurun_out/gf16_bench.json")
    a = ap.parse_args()
    ctx = qf.default_context()
    res = {}
    rng = np.random.default_rng(1)

    for name, k, r, L, G, e in (("batched_k64_r16", 64, 16, 1200, a.G, 16), ("extreme_k1024_n2048", 1024, 1024, 1200, 1, 512),
                                ("extreme_k1024_x16", 1024, 1024, 1200, 16, 512)):
        rs = _r16(L)
        src = torch.randint(0, 256, (G * k * rs,), dtype=torch.uint8, device="cuda")
        rep = torch.empty(G * r * rs, dtype=torch.uint8, device="cuda")

        def enc():
            qf.encode16_batch(src, rep, k, r, L, src_row_stride=rs, src_gen_stride=k * rs, rep_row_stride=rs,
                              rep_gen_stride=r * rs, G=G)

        wall, kt = timed(ctx, enc, a.reps)
        kms = sum(ms for _, ms in kt.values())
        res[name + "/encode16"] = {"k": k, "r": r, "L": L, "G": G, "wall_ms": round(wall, 3), "kernels": kt,
                                   "GiBps_alg": round(G * (k + r) * L / (kms / 1e3) / 2**30, 1)}
        # decode: the first k rows = k - e sources + e repairs, Cauchy rows
        max_rows = k
        arr = np.zeros((G, k), np.uint16)
        for g in range(G):
            er = rng.choice(k, e, replace=False)
            keep = np.setdiff1d(np.arange(k), er)
            row = np.concatenate([keep, k + rng.permutation(r)[:e]])
            rng.shuffle(row)
            arr[g] = row
        # rows: gather sources/repairs on the device
        rows = torch.empty(G * k * rs, dtype=torch.uint8, device="cuda")
        src3, rep3, rows3 = (t.view(G, -1, rs) for t in (src, rep, rows))
        ai = torch.from_numpy(arr.astype(np.int64)).to("cuda")
        for g in range(G):
            sel = ai[g]
            rows3[g] = torch.where((sel < k)[:, None], src3[g][sel.clamp(max=k - 1)], rep3[g][(sel - k).clamp(min=0)])
        t_idx = torch.from_numpy(arr.view(np.int16)).to("cuda")
        emax = min(k, r)
        rec = torch.empty(G * emax * rs, dtype=torch.uint8, device="cuda")
        ri = torch.empty(G * emax, dtype=torch.int16, device="cuda")
        nrec = torch.empty(G, dtype=torch.int32, device="cuda")
        st = torch.empty(G, dtype=torch.int32, device="cuda")

        def dec():
            qf.decode16_batch(rows, t_idx, rec, ri, nrec, st, k, r, L, max_rows=max_rows, row_stride=rs,
                              rows_gen_stride=k * rs, rec_row_stride=rs, rec_gen_stride=emax * rs, G=G)

        wall, kt = timed(ctx, dec, a.reps)
        assert (st == 0).all().item() and (nrec == e).all().item()
        # spot-check one generation against the sources
        g = G - 1
        er = sorted(set(range(k)) - set(int(x) for x in arr[g] if x < k))
        got = rec.view(G, emax, rs)[g, :e, :L]
        want = src3[g][torch.tensor(er, device="cuda")][:, :L]
        assert torch.equal(got, want)
        kms = sum(ms for _, ms in kt.values())
        res[name + "/decode16"] = {"k": k, "r": r, "L": L, "G": G, "erasures": e, "wall_ms": round(wall, 3),
                                   "kernels": kt, "GiBps_alg": round(G * (k + e) * L / (kms / 1e3) / 2**30, 1)}
        if k >= 1024:   # the FFT variants (QF_OPT_GF16_FFT_BS): bit planes always (2), radix 4 (3), log / Zech (0)
            for v in (2, 3, 0):
                qf.set_default_options(gf16_fft_bs=v)
                wall, kt = timed(ctx, enc, a.reps)
                kms = sum(ms for _, ms in kt.values())
                res[f"{name}/encode16_bs{v}"] = {"wall_ms": round(wall, 3), "kernels": kt,
                                                 "GiBps_alg": round(G * (k + r) * L / (kms / 1e3) / 2**30, 1)}
                wall, kt = timed(ctx, dec, a.reps)
                assert (st == 0).all().item() and torch.equal(rec.view(G, emax, rs)[g, :e, :L], want)
                kms = sum(ms for _, ms in kt.values())
                res[f"{name}/decode16_bs{v}"] = {"wall_ms": round(wall, 3), "kernels": kt,
                                                 "GiBps_alg": round(G * (k + e) * L / (kms / 1e3) / 2**30, 1)}
            qf.reset_default_options()
        print(name, json.dumps({kk: v for kk, v in res.items() if kk.startswith(name)}), flush=True)
        del src, rep, rows, rec

    # encode only: more power-of-two windows (additive FFT), and the general
    # k_matvec16 kernel on the same inputs (gf16_fft = 0) for comparison
    for name, k, r, L, G in (("extreme_k1024_x64", 1024, 1024, 1200, 64), ("extreme_k4096_n8192", 4096, 4096, 1200, 1),
                             ("k128_r32_x2048", 128, 32, 1200, 2048), ("extreme_k1024_x16", 1024, 1024, 1200, 16)):
        rs = _r16(L)
        src = torch.randint(0, 256, (G * k * rs,), dtype=torch.uint8, device="cuda")
        rep = torch.empty(G * r * rs, dtype=torch.uint8, device="cuda")

        def enc():
            qf.encode16_batch(src, rep, k, r, L, src_row_stride=rs, src_gen_stride=k * rs, rep_row_stride=rs,
                              rep_gen_stride=r * rs, G=G)

        for mode in ("fft", "matvec"):
            qf.set_default_options(gf16_fft=1 if mode == "fft" else 0)
            if mode == "matvec" and k > 1024:
                continue
            wall, kt = timed(ctx, enc, a.reps)
            kms = sum(ms for _, ms in kt.values())
            res[f"{name}/encode16_{mode}"] = {"k": k, "r": r, "L": L, "G": G, "wall_ms": round(wall, 3),
                                             "kernels": kt,
                                             "GiBps_alg": round(G * (k + r) * L / (kms / 1e3) / 2**30, 1)}
            if mode == "fft":
                out_fft = rep.clone()
            else:
                res[f"{name}/encode16_{mode}"]["same_bytes_as_fft"] = bool(
                    torch.equal(rep.view(G, r, rs)[:, :, :L], out_fft.view(G, r, rs)[:, :, :L]))
            print(name, mode, json.dumps(res[f"{name}/encode16_{mode}"]), flush=True)
        qf.reset_default_options()
        del src, rep

    # oracle single thread, one generation of each shape (CPU reference point)
    for name, k, r, L in (("batched_k64_r16", 64, 16, 1200), ("extreme_k1024_n2048", 1024, 1024, 1200)):
        s = rng.integers(0, 256, (k, L), dtype=np.uint8)
        t0 = time.perf_counter()
        oracle.encode16(s, r if k == 64 else 64)  # extreme: 64 of the 1024 repairs, scaled
        dt = time.perf_counter() - t0
        scale = 1 if k == 64 else r / 64
        res[name + "/oracle_encode16_1thread"] = {"ms_per_generation": round(dt * scale * 1e3, 2),
                                                  "MiBps_alg": round((k + r) * L / (dt * scale) / 2**20, 2)}
    Path(a.out).parent.mkdir(exist_ok=True)
    Path(a.out).write_text(json.dumps(res, indent=1))
    print(json.dumps({k: v.get("GiBps_alg", v.get("MiBps_alg")) for k, v in res.items()}))


if __name__ == "__main__":
    main()
