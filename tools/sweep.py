"""Kernel-variant sweep on one GPU (diagnostic tool, not the benchmark).

Times k_combine_uniform (encode) for several output widths R and prefetch
depths PD, the decode pair for several PD, and a device copy of the same
byte count as a bandwidth reference.  Variants are selected per call with
the context's kernel-path options (qf_ctx_set_option: bitsliced, encode_v,
encode_pd, decode_pd) -- the QF_* environment variables are read only when a
context is created, so setting them here would not reach the library."""
import json
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import bench  # noqa: E402
from quicfuscate_amd import _lib as L  # noqa: E402
from quicfuscate_amd import fec  # noqa: E402


def timeit(fn, reps=5, warm=2):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return float(np.median(ts)), float(np.min(ts))


def main():
    G = int(os.environ.get("SWEEP_G", "65536"))
    k, Lb = 64, 1200
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    # run everything on torch's default stream: the context must use it too
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    ctx = fec.Context(0, s.cuda_stream)
    lib = L._lib()
    res = {}
    defaults = {n: ctx.option(n) for n in ("bitsliced", "encode_v", "encode_pd", "decode_pd")}
    src = torch.empty(G * k * Lb, dtype=torch.uint8, device=dev)
    L.check(lib.qf_fill_splitmix_dev(ctx.handle, src.data_ptr(), src.numel(), bench.SEED, 0))
    rep = torch.empty(G * 16 * Lb, dtype=torch.uint8, device=dev)
    dst = torch.empty_like(src)
    ms, mn = timeit(lambda: dst.copy_(src))
    res["copy_src_GBps"] = round(2 * src.numel() / (mn / 1e3) / 1e9, 1)
    for r in (10, 16):
        ctx.set_option("bitsliced", defaults["bitsliced"])
        f = lambda: fec.encode_batch(src, rep, k, r, Lb, src_row_stride=Lb, src_gen_stride=k * Lb,
                                     rep_row_stride=Lb, rep_gen_stride=r * Lb, G=G, ctx=ctx)
        ms, mn = timeit(f)
        byt = G * (k + r) * Lb
        res[f"enc_r{r}_bitsliced"] = {"ms": round(mn, 4), "GBps": round(byt / (mn / 1e3) / 1e9, 1)}
        print(f"enc r={r} bitsliced: {res[f'enc_r{r}_bitsliced']}", flush=True)
    ctx.set_option("bitsliced", 0)
    for r in (1, 16):
        for V, PD in ((1, 1), (1, 2)):
            if r >= 9 and V == 2:
                continue
            ctx.set_option("encode_v", V)
            ctx.set_option("encode_pd", PD)
            f = lambda: fec.encode_batch(src, rep, k, r, Lb, src_row_stride=Lb, src_gen_stride=k * Lb,
                                         rep_row_stride=Lb, rep_gen_stride=r * Lb, G=G, ctx=ctx)
            ms, mn = timeit(f)
            byt = G * (k + r) * Lb
            res[f"enc_r{r}_V{V}_PD{PD}"] = {"ms": round(mn, 4), "GBps": round(byt / (mn / 1e3) / 1e9, 1),
                                           "src_GiBps": round(G * k * Lb / (mn / 1e3) / 2**30, 1)}
            print(f"enc r={r} V={V} PD={PD}: {res[f'enc_r{r}_V{V}_PD{PD}']}", flush=True)
    for n in ("encode_v", "encode_pd", "bitsliced"):
        ctx.set_option(n, defaults[n])
    fec.encode_batch(src, rep, k, 16, Lb, src_row_stride=Lb, src_gen_stride=k * Lb, rep_row_stride=Lb,
                     rep_gen_stride=16 * Lb, G=G, ctx=ctx)
    del dst
    e, r = 13, 16
    erased = bench.erasure_plan(G, k, e, 1)
    aidx = bench.arrival_index(erased, k, r)
    n = aidx.shape[1]
    rows = torch.empty(G * n * Lb, dtype=torch.uint8, device=dev)
    sv, rv, ov = src.view(G, k, Lb), rep.view(G, r, Lb), rows.view(G, n, Lb)
    at = torch.from_numpy(aidx.astype(np.int64)).to(dev)
    for g0 in range(0, G, 4096):
        g1 = min(G, g0 + 4096)
        both = torch.cat([sv[g0:g1], rv[g0:g1]], dim=1)
        gi = torch.arange(g1 - g0, device=dev)[:, None].expand(-1, n)
        ov[g0:g1] = both[gi, at[g0:g1]]
    ridx = torch.from_numpy(aidx.view(np.int16)).to(dev)
    rec = torch.empty(G * 16 * Lb, dtype=torch.uint8, device=dev)
    reci = torch.empty(G * 16, dtype=torch.int16, device=dev)
    nrec = torch.empty(G, dtype=torch.int32, device=dev)
    st = torch.empty(G, dtype=torch.int32, device=dev)
    for PD in (1, 2, 3):
        ctx.set_option("decode_pd", PD)
        f = lambda: fec.decode_batch(rows, ridx, rec, reci, nrec, st, k, r, Lb, max_rows=n, row_stride=Lb,
                                     rows_gen_stride=n * Lb, rec_row_stride=Lb, rec_gen_stride=16 * Lb, G=G, ctx=ctx)
        ms, mn = timeit(f)
        byt = G * (k * Lb + e * k + e * Lb)
        ok = bool((st == 0).all().item())
        res[f"dec_PD{PD}"] = {"ms": round(mn, 4), "GBps": round(byt / (mn / 1e3) / 1e9, 1), "ok": ok}
        print(f"dec PD={PD}: {res[f'dec_PD{PD}']}", flush=True)
    ctx.set_option("decode_pd", defaults["decode_pd"])
    print(json.dumps(res))


if __name__ == "__main__":
    main()
