#!/usr/bin/env python3
"""Latency of one generation's decode through the decoder object (the
per-connection path: Decoder::add_packet completing a generation,
decoder.rs:678-783): the add_packet call that brings the k-th row, split into
the library's kernels (context HIP events) and the rest (uploads, syncs,
downloads, host assembly).

    python tools/bench_dec_latency.py [--reps 50] [--out gpurun_out/dec_latency.json]
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

# (k, n) of the adaptive modes that decode on GF(2^8) (adaptive.rs:124-153)
SHAPES = [("Light", 16, 17, 1), ("Normal", 64, 74, 10), ("Medium", 128, 167, 26)]


def main():
    import torch

    from quicfuscate_amd import fec as qf
    from tests import oracle_py as oracle   # repairs only (test data)

    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--L", type=int, default=1024)
    ap.add_argument("--out", default="gpurun_out/dec_latency.json")
    a = ap.parse_args()
    assert torch.cuda.is_available()
    ctx = qf.default_context()
    res = {}
    for name, k, n, e in SHAPES:
        r = n - k
        rng = np.random.default_rng(k)
        src = rng.integers(0, 256, (k, a.L), dtype=np.uint8)
        C = oracle.cauchy(k, r)
        rep = oracle.encode(src, r)
        lost = set(range(0, k, max(1, k // e)))
        lost = set(sorted(lost)[:e])
        pk = [qf.Packet(i, bytearray(src[i].tobytes()), a.L, True) for i in range(k) if i not in lost]
        pk += [qf.Packet(10_000 + j, bytearray(rep[j].tobytes()), a.L, False, bytes(C[j]), k) for j in range(e)]
        walls, kern = [], {}
        # first pass: wall time only; second pass: per-kernel event times
        for it in range(2 * a.reps + 3):
            prof = it >= a.reps + 3
            dec = qf.Decoder(k, max_len=a.L)
            for p in pk[:-1]:
                dec.add_packet(p)
            ctx.sync()
            if prof:
                ctx.profile(True)
            t0 = time.perf_counter()
            assert dec.add_packet(pk[-1])
            t1 = time.perf_counter()
            if prof:
                for kn, (c, ms) in ctx.kernel_times().items():
                    kern[kn] = kern.get(kn, 0.0) + ms
                ctx.profile(False)
            elif it >= 3:
                walls.append((t1 - t0) * 1e6)
            got = np.stack([np.frombuffer(p.payload(), np.uint8) for p in dec.get_decoded_packets()])
            assert (got == src).all()
        res[name] = {"k": k, "r": r, "e": e, "L": a.L, "decode_call_us_median": round(float(np.median(walls)), 1),
                     "decode_call_us_min": round(float(np.min(walls)), 1),
                     "kernels_us_per_call": {kn: round(v / a.reps * 1e3, 1) for kn, v in kern.items()}}
        print(name, res[name], flush=True)
    Path(a.out).parent.mkdir(exist_ok=True)
    Path(a.out).write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
