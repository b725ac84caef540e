"""Multi-rank bench logic on CPU (gloo, world size 2): generation sharding,
distinct per-rank payload, and the max-over-ranks reduction bench.py uses
(independent generations, no data-path collective)."""
import os
import socket

import numpy as np
import pytest

import bench


def test_shards_partition_generations():
    for total in (1, 7, 65536, 156250):
        for world in (1, 2, 4, 8):
            ranges = [bench.shard_generations(total, r, world) for r in range(world)]
            assert ranges[0][0] == 0 and ranges[-1][1] == total
            for (a, b), (c, d) in zip(ranges, ranges[1:]):
                assert b == c and a <= b
            sizes = [b - a for a, b in ranges]
            assert max(sizes) - min(sizes) <= 1


def test_xor_fold():
    import functools
    import operator

    import torch

    x = torch.arange(1001, dtype=torch.int64) * 0x9E3779B97F4A7C15 % (1 << 62)
    assert bench.xor_fold(torch, x.view(torch.uint8)) == functools.reduce(operator.xor, x.tolist())


def test_payload_offsets_distinct_and_disjoint():
    G, k, L = 1000, 64, 1200
    offs = [bench.payload_word_offset(r, G, k, L) for r in range(8)]
    words = G * k * L // 8
    assert all(b - a == words for a, b in zip(offs, offs[1:]))


def test_erasure_plan_seeded_and_arrival_order():
    e1 = bench.erasure_plan(50, 64, 13, 7)
    e2 = bench.erasure_plan(50, 64, 13, 7)
    assert (e1 == e2).all() and e1.shape == (50, 13)
    assert all(len(set(row)) == 13 and list(row) == sorted(row) for row in e1)
    a = bench.arrival_index(e1, 64, 16)
    assert a.shape == (50, 64 - 13 + 16)
    for g in range(50):
        surv = [i for i in range(64) if i not in set(e1[g])]
        assert list(a[g]) == surv + list(range(64, 80))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = bench.shard_generations(1000, rank, world)
    # rank-dependent "timings"; rank 1 reports a failed verification
    vals = [10.0 + rank, 3.0 * (rank + 1), 7.0 - rank, float(rank == 1)]
    out = bench.reduce_max(torch, dist, vals, world, "cpu")
    folds = bench.gather_folds(torch, dist, (0xF000000000000000 | rank), world, "cpu")
    assert folds == [0xF000000000000000, 0xF000000000000001]
    assert bench.gather_flags(torch, dist, rank == 0, world, "cpu") == [1, 0]
    # rank 0's run descriptor + Cauchy matrix reach every rank (host-only ABI call)
    from quicfuscate_amd import _lib as L

    assert bench.broadcast_descriptor(torch, dist, L._lib(), 64, 16, 1200, 1000, 13, world, "cpu")
    dist.barrier()
    dist.destroy_process_group()
    q.put((rank, lo, hi, out))


@pytest.mark.timeout(120)
def test_gloo_world2_max_over_ranks():
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=100) for _ in procs)
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    assert [(r, lo, hi) for r, lo, hi, _ in res] == [(0, 0, 500), (1, 500, 1000)]
    for _, _, _, out in res:
        assert np.allclose(out, [11.0, 6.0, 7.0, 1.0])


def _halo_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist

    from quicfuscate_amd import stream_shard as ss

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        P, k, stride = 37, 8, 16
        g = torch.arange(P * stride, dtype=torch.int64).view(P, stride).remainder(251).to(torch.uint8)
        lo, hi = ss.packet_range(P, rank, world)
        ext = ss.halo_exchange(torch, dist, g[lo:hi].clone(), k, rank, world)
        first, nwin = ss.local_windows(lo, hi, k)
        wins = [ext[t - lo: t - lo + k].clone() for t in range(first, first + nwin)]
        ok = all(torch.equal(w, g[t - k + 1: t + 1]) for w, t in zip(wins, range(first, first + nwin)))
        q.put((rank, lo, hi, first, nwin, ok))
    finally:
        dist.destroy_process_group()


def test_sliding_halo_exchange_gloo():
    """Sliding-window sharding: after the k - 1 packet halo
    from the previous rank, every rank's windows equal the global stream's,
    and the ranks' windows together cover every window exactly once."""
    import multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 3
    procs = [ctx.Process(target=_halo_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for *_, ok in res)
    ends = [t for _, lo, hi, first, nwin, _ in res for t in range(first, first + nwin)]
    assert ends == list(range(8 - 1, 37))


def _short_halo_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist

    from quicfuscate_amd import stream_shard as ss

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        k = 8
        n = 3 if rank == 0 else 10          # rank 0 cannot send a k - 1 = 7 packet halo
        try:
            ss.halo_exchange(torch, dist, torch.zeros((n, 16), dtype=torch.uint8), k, rank, world)
            q.put((rank, "no error"))
        except ValueError:
            q.put((rank, "raised"))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_halo_short_shard_raises_on_every_rank():
    """A shard smaller than the halo is an error on ALL ranks before any
    send / recv (a lone raise would leave the successor blocked in recv)."""
    import multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_short_halo_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=100) for _ in procs)
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    assert res == [(0, "raised"), (1, "raised")]
