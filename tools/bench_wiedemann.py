#!/usr/bin/env python3
"""Timing of the k > 256 GF(2^8) decoder (Wiedemann strategy):
per shape, the wall time of the add_packet call that completes the
generation (row upload + device solve + payload pass + download of the
recovered rows), and of the whole generation's add_packet loop.

    python tools/bench_wiedemann.py --out gpurun_out/wiedemann_bench.json

Run it under rocprofv3 --kernel-trace --stats for the per-kernel split."""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))

SHAPES = [(260, 2, 1200), (512, 13, 1200), (1024, 16, 1200), (4096, 40, 1200), (4096, 128, 1200),
          (2048, 256, 1200)]


def main():
    import torch

    from quicfuscate_amd import fec as qf
    from tests import oracle_py as oracle   # test-data generation only (the repairs)

    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out", default="gpurun_out/wiedemann_bench.json")
    a = ap.parse_args()
    assert torch.cuda.is_available()
    res = {}
    for k, e, L in SHAPES:
        rng = np.random.default_rng(k + e)
        src = rng.integers(0, 256, (k, L), dtype=np.uint8)
        lost = set(rng.choice(k, e, replace=False).tolist())
        coef = rng.integers(1, 256, (e, k), dtype=np.uint8)
        rep = oracle.encode(src, e, coef)
        pk = [qf.Packet(i, bytearray(src[i].tobytes()), L, True) for i in range(k) if i not in lost]
        pk += [qf.Packet(10_000 + j, bytearray(rep[j].tobytes()), L, False, bytes(coef[j]), k) for j in range(e)]
        last, whole = [], []
        for _ in range(a.reps):
            dec = qf.Decoder(k, max_len=L)
            t0 = time.perf_counter()
            for p in pk[:-1]:
                dec.add_packet(p)
            t1 = time.perf_counter()
            assert dec.add_packet(pk[-1])
            t2 = time.perf_counter()
            last.append((t2 - t1) * 1e3)
            whole.append((t2 - t0) * 1e3)
            got = np.stack([np.frombuffer(p.payload(), np.uint8) for p in dec.get_decoded_packets()])
            assert (got == src).all()
        res[f"k{k}_e{e}_L{L}"] = {"k": k, "e": e, "L": L, "decode_call_ms": round(min(last), 3),
                                  "generation_ms": round(min(whole), 3), "verified": True}
        print(res[f"k{k}_e{e}_L{L}"], flush=True)
    Path(a.out).parent.mkdir(exist_ok=True)
    Path(a.out).write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
