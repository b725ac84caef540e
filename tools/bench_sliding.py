#!/usr/bin/env python3
"""Sliding-window encode of one packet stream sharded over ranks:
each rank owns a contiguous packet range, receives the k - 1 packet halo from
the previous rank (send/recv: RCCL over xGMI), and encodes one window per own
packet (adaptive.rs:519-562) in one batched call.  Timed per step: halo +
encode, max over ranks.  value = stream payload bytes of all ranks / s.

  python tools/bench_sliding.py [--packets 200000] [--k 64 --r 10 --L 1200]
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 tools/bench_sliding.py
  (QF_BENCH_BACKEND=gloo rehearses several ranks on one GPU)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))


def main():
    import torch
    import torch.distributed as dist

    ap = argparse.ArgumentParser()
    ap.add_argument("--packets", type=int, default=200000, help="packets per rank")
    ap.add_argument("--k", type=int, default=64)
    ap.add_argument("--r", type=int, default=10)
    ap.add_argument("--L", type=int, default=1200)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    a = ap.parse_args()
    rank, world = int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("QF_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    from quicfuscate_amd import _lib as L
    from quicfuscate_amd import fec
    from quicfuscate_amd import stream_shard as ss

    dev = torch.device("cuda", local)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    ctx = fec.Context(local, stream.cuda_stream)
    k, r, Lb = a.k, a.r, a.L
    P = a.packets * world
    lo, hi = ss.packet_range(P, rank, world)
    stride = (Lb + 15) // 16 * 16
    Lr = (Lb + 127) // 128 * 128
    rows = torch.empty((hi - lo, stride), dtype=torch.uint8, device=dev)
    L.check(L._lib().qf_fill_splitmix_dev(ctx.handle, rows.data_ptr(), rows.numel(), 0x51464543,
                                           lo * stride // 8), "fill")
    _, nwin = ss.local_windows(lo, hi, k)
    rep = torch.empty(max(1, nwin) * r * Lr, dtype=torch.uint8, device=dev)

    def step():
        ext = ss.halo_exchange(torch, dist, rows, k, rank, world)
        ss.encode_sliding_local(ext, lo, hi, k, r, Lb, rep, rep_row_stride=Lr, zero_tail=True, ctx=ctx)

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = (time.perf_counter() - t0) / a.steps
    t = torch.tensor([dt], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    if rank == 0:
        print(json.dumps({"metric": "sliding-window encode GiB/s of stream payload", "value": round(P * Lb / dt / 2**30, 2),
                          "unit": "GiB/s", "n_gpus": world, "ms_per_step": round(dt * 1e3, 3), "packets": P,
                          "windows_per_s": round((P - (k - 1)) / dt, 0), "config": {"k": k, "r": r, "L": Lb,
                          "halo_packets": k - 1, "backend": backend if world > 1 else "none"}}))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
