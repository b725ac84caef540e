"""Parity at BASELINE.json's full sizes, through size-independent properties.

The CPU oracle cannot run millions of generations in a test, so the full
sizes are checked by properties that hold at any size, plus oracle parity on
a seeded sample of generations:

* configs[1] + configs[2] (the bench workload: k=64, r=16, L=1200, 65,536
  generations, 13 of 64 sources erased per generation): encode -> erase ->
  decode returns the erased sources bit-exact, on both Cauchy decode paths
  (the fused kernel and QF_DECODE_SYN=1), and sampled generations' repairs
  equal the oracle's (decoder.rs:172-275);
* configs[3] (10 M packets per GPU, generations sharded over 8 ranks):
  encoding the 8 rank slices separately gives the same bytes as one batch
  over all 156,250 generations (independent generations: the multi-GPU path
  has no data-path collective), and the code is GF(2)-linear
  (enc(a ^ b) == enc(a) ^ enc(b)) over the whole batch.

Inputs are splitmix64 bytes filled on the device (the bench's generator)."""
import numpy as np
import pytest

import bench

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _bit_sliced_encode(qf):
    # these tests pin the bit-sliced kernels (and their zero tails) at small
    # G; the small-batch kernel has its own cases (test_gpu_encode.py)
    qf.set_default_options(encode_small=0)

K, R, L = 64, 16, 1200
SEED = 0x51464543


def _fill(torch, qf, n, seed, word_offset=0):
    from quicfuscate_amd import _lib as Lb

    ctx = qf.default_context()
    buf = torch.empty(n, dtype=torch.uint8, device="cuda")
    Lb.check(Lb._lib().qf_fill_splitmix_dev(ctx.handle, buf.data_ptr(), n, seed, word_offset), "fill")
    return buf


def _sync(torch, qf):
    qf.default_context().sync()
    torch.cuda.synchronize()


def _oracle_sample(oracle, srcv, repv, G, n, seed):
    """Repairs of n seeded generations against the oracle, bit-exact."""
    rng = np.random.default_rng(seed)
    for g in rng.choice(G, size=n, replace=False).tolist():
        want = oracle.encode(srcv[g].cpu().numpy(), R, L=L)
        got = repv[g, :, :L].cpu().numpy()
        assert np.array_equal(got, want), f"generation {g}: repairs differ from the oracle"


@pytest.mark.parametrize("path", ["fused", "syndrome"])
def test_bench_workload_full_size_round_trip(qf, oracle, gpu_ctx, path, monkeypatch):
    import torch

    if path == "syndrome":
        qf.set_default_options(decode_path=1)
    G, e = 65536, 13
    Lr = (L + 127) // 128 * 128           # the bench's pool-block repair rows
    src = _fill(torch, qf, G * K * L, SEED)
    rep = torch.full((G * R * Lr,), 0xA5, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    qf.encode_batch(src, rep, K, R, L, src_row_stride=L, src_gen_stride=K * L, rep_row_stride=Lr,
                    rep_gen_stride=R * Lr, G=G, zero_tail=True)
    _sync(torch, qf)
    srcv, repv = src.view(G, K, L), rep.view(G, R, Lr)
    assert bool((repv[:, :, L:] == 0).all()), "zero tails"
    _oracle_sample(oracle, srcv, repv, G, 24, SEED + 1)

    erased = bench.erasure_plan(G, K, e, SEED + 2)
    aidx = bench.arrival_index(erased, K, R)
    n_slots = aidx.shape[1]
    rows = torch.empty(G * n_slots * L, dtype=torch.uint8, device="cuda")
    rowsv = rows.view(G, n_slots, L)
    aidx_t = torch.from_numpy(aidx.astype(np.int64)).cuda()
    for g0 in range(0, G, 4096):
        g1 = min(G, g0 + 4096)
        both = torch.cat([srcv[g0:g1], repv[g0:g1, :, :L]], dim=1)
        gi = torch.arange(g1 - g0, device="cuda")[:, None].expand(-1, n_slots)
        rowsv[g0:g1] = both[gi, aidx_t[g0:g1]]
        del both
    row_index = torch.from_numpy(aidx.view(np.int16)).cuda()
    rec = torch.full((G * R * L,), 0x5A, dtype=torch.uint8, device="cuda")
    rec_index = torch.full((G * R,), -1, dtype=torch.int16, device="cuda")
    n_rec = torch.empty(G, dtype=torch.int32, device="cuda")
    status = torch.full((G,), 99, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    qf.decode_batch(rows, row_index, rec, rec_index, n_rec, status, K, R, L, max_rows=n_slots, row_stride=L,
                    rows_gen_stride=n_slots * L, rec_row_stride=L, rec_gen_stride=R * L, G=G)
    _sync(torch, qf)
    assert bool((status == 0).all()), "status"
    assert bool((n_rec == e).all()), "recovered count"
    er_t = torch.from_numpy(erased).cuda()
    assert bool((rec_index.view(G, R)[:, :e].long() == er_t).all()), "recovered indices"
    gi = torch.arange(G, device="cuda")[:, None].expand(-1, e)
    assert bool((rec.view(G, R, L)[:, :e] == srcv[gi, er_t]).all()), "recovered bytes"


def test_ten_million_packets_sharded_and_linear(qf, oracle, gpu_ctx):
    import torch

    G = 10_000_000 // K                   # 156,250 generations = 10 M source packets
    world = 8
    a = _fill(torch, qf, G * K * L, SEED + 3)
    b = _fill(torch, qf, G * K * L, SEED + 4)
    shape = dict(src_row_stride=L, src_gen_stride=K * L, rep_row_stride=L, rep_gen_stride=R * L)

    def enc(src, rep, g0=0, g1=G):
        torch.cuda.synchronize()          # torch-made inputs are complete (the library has its own stream)
        qf.encode_batch(src[g0 * K * L:], rep[g0 * R * L:], K, R, L, G=g1 - g0, **shape)

    ra = torch.empty(G * R * L, dtype=torch.uint8, device="cuda")
    enc(a, ra)
    # the same job as 8 rank slices (bench.shard_generations), each its own launch
    rs = torch.full_like(ra, 0xA5)
    for rank in range(world):
        lo, hi = bench.shard_generations(G, rank, world)
        enc(a, rs, lo, hi)
    _sync(torch, qf)
    assert torch.equal(ra, rs), "sharded encode differs from the single batch"
    del rs
    _oracle_sample(oracle, a.view(G, K, L), ra.view(G, R, L), G, 16, SEED + 5)

    rb = torch.empty_like(ra)
    enc(b, rb)
    ab = torch.bitwise_xor(a, b)
    del b
    rab = torch.empty_like(ra)
    enc(ab, rab)
    _sync(torch, qf)
    assert torch.equal(rab, torch.bitwise_xor(ra, rb)), "enc(a ^ b) != enc(a) ^ enc(b)"
