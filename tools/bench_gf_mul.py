#!/usr/bin/env python3
"""The reference's benches/gf_mul.rs, gf_bitslice.rs and gf_mul_slice_bench.rs
on the MI355X: element-wise GF(2^8) products a[i] * b[i] (gf_tables.rs:255
gf_mul_slice; gf_mul per element), device resident, from the benches' 1 KiB
up to 1 GiB, beside the oracle's scalar table loop.  Algorithmic bytes 3n
(two inputs, one output).

    python tools/bench_gf_mul.py [--out gpurun_out/gf_mul.json]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))


def main():
    import torch

    from quicfuscate_amd import _lib as L
    from quicfuscate_amd import fec as qf
    from tests import oracle_py as oracle

    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/gf_mul.json")
    a = ap.parse_args()
    ctx = qf.default_context()
    lib = L._lib()
    res = {}
    for n in (1024, 1 << 20, 1 << 26, 1 << 30):
        x = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda")
        y = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda")
        out = torch.empty_like(x)
        reps = 200 if n <= 1 << 20 else 20

        def call():
            L.check(lib.qf_gf256_mul_slice_dev(ctx.handle, x.data_ptr(), y.data_ptr(), out.data_ptr(), n), "slice")

        call()
        ctx.sync()
        ctx.profile(True)
        t0 = time.perf_counter()
        for _ in range(reps):
            call()
        ctx.sync()
        wall = (time.perf_counter() - t0) / reps
        kt = ctx.kernel_times()
        ctx.profile(False)
        kms = sum(ms for _, ms in kt.values()) / reps
        # parity on a sample against the table
        idx = torch.randint(0, n, (4096,), device="cuda")
        xs, ys, os_ = (t[idx].cpu().numpy() for t in (x, y, out))
        tab = oracle.mul_table_full()
        assert (tab[xs, ys] == os_).all()
        res[str(n)] = {"bytes": n, "kernel_us": round(kms * 1e3, 2), "call_us": round(wall * 1e6, 2),
                       "GBps_alg": round(3 * n / (kms / 1e3) / 1e9, 1), "frac_of_8TBps": round(3 * n / (kms / 1e3) / 8e12, 3)}
        print(n, res[str(n)], flush=True)
    # the benches' CPU work: 1024 table products (oracle, numpy-vectorised and scalar loop)
    tab = oracle.mul_table_full()
    av = np.arange(1024, dtype=np.uint8)
    bv = (255 - np.arange(1024)).astype(np.uint8)
    t0 = time.perf_counter()
    for _ in range(100):
        acc = 0
        for i in range(1024):
            acc ^= int(tab[av[i], bv[i]])
    res["oracle_scalar_1024_us"] = round((time.perf_counter() - t0) / 100 * 1e6, 1)
    Path(a.out).parent.mkdir(exist_ok=True)
    Path(a.out).write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
