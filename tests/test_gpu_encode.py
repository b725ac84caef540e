"""Encode parity on the MI355X: k_combine_uniform vs the CPU oracle.

Bit-exact comparison of every repair byte, plus the bytes around each repair
row (the library must write exactly L bytes per row)."""
import hashlib
import json
import os
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _bit_sliced_encode(qf):
    # these tests pin the bit-sliced kernels (and their zero tails) at small
    # G; the small-batch kernel has its own cases (test_gpu_encode.py)
    qf.set_default_options(encode_small=0)


GOLDEN = json.loads((Path(__file__).parent / "golden" / "golden.json").read_text())


def _r16(x):
    return (x + 15) // 16 * 16


def run_encode(qf, src_np, k, r, L, G, rs, gs, rrs, rgs, coeff=None, zero_tail=False):
    import torch

    dev = torch.device("cuda")
    src = torch.from_numpy(src_np).to(dev)
    rep = torch.full((G * rgs + 64,), 0xA5, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    qf.encode_batch(src, rep, k, r, L, src_row_stride=rs, src_gen_stride=gs, rep_row_stride=rrs,
                    rep_gen_stride=rgs, G=G, coeff=coeff, zero_tail=zero_tail)
    qf.default_context().sync()
    return rep.cpu().numpy()


CASES = [
    # k, r, L, G
    (64, 16, 1200, 37),    # the benchmark shape
    (16, 16, 1200, 5),
    (16, 1, 1200, 9),      # Light mode params_for(Light,16) = (16,17)
    (4, 2, 8, 3),          # tests/fec.rs make_packet shape
    (7, 5, 33, 11),        # odd k, odd r, tail unit
    (1, 1, 16, 2),
    (3, 3, 1, 130),        # 1-byte packets, many generations per wave
    (255, 1, 64, 2),       # largest k
    (200, 56, 48, 1),      # k + r = 256 (largest valid), 4 passes
    (64, 40, 100, 3),      # r > 16 -> passes of 16
    (96, 15, 9000, 2),     # jumbo payload (Normal ratio 1.15: r = 15 at k = 96)
    (63, 16, 1201, 7),     # k % 4 = 3, L % 16 = 1
    # shapes with a bit-sliced Cauchy kernel (bs_codegen.py): whole and half
    # 32-byte chunks, several generations per wave
    (32, 16, 96, 10),
    (64, 10, 64, 21),
    (16, 16, 80, 13),
    (64, 16, 1216, 11),
]


ZERO_TAIL_CASES = [
    # k, r, L, G, repair row stride, repair generation stride
    (64, 16, 1200, 41, 1280, 16 * 1280),         # the benchmark layout
    (64, 16, 1200, 9, 1296, 16 * 1296 + 48),     # room beyond the tail: untouched
    (16, 1, 1200, 17, 1200, 1280),               # r = 1: the tail fits the generation
    (32, 16, 96, 23, 128, 16 * 128),             # 6 units -> 8: two padding lanes per row
    (64, 10, 64, 50, 64, 640),                   # 4 units -> 8, no room for the tail: plain path
    (64, 16, 1200, 5, 1216, 16 * 1216),          # stride too short for the tail: plain path
    (7, 5, 33, 11, 48, 5 * 48),                  # no bit-sliced kernel: flag ignored
]


@pytest.mark.parametrize("k,r,L,G,rrs,rgs", ZERO_TAIL_CASES)
def test_encode_zero_tail(qf, oracle, gpu_ctx, k, r, L, G, rrs, rgs):
    """QF_ENCODE_ZERO_TAIL: repairs bit-exact; bytes [L, round_up(L, 128)) of
    a row are zero or untouched (zero exactly when the tail fits the layout
    and a bit-sliced kernel runs); nothing beyond them is written."""
    rng = np.random.default_rng(k + r + L + G)
    rs = _r16(L)
    gs = k * rs
    src = rng.integers(0, 256, G * gs, dtype=np.uint8)
    rep = run_encode(qf, src, k, r, L, G, rs, gs, rrs, rgs, zero_tail=True)
    tail = (L // 16 + 7) // 8 * 128 if L % 16 == 0 else L
    fits = (r == 1 or rrs >= tail) and rgs >= (r - 1) * rrs + tail
    bs_shape = (k, r) in {(64, 16), (64, 10), (32, 16), (16, 16), (16, 1)} and L % 16 == 0 and L >= 32
    if not fits:
        tail = L
    for g in range(G):
        rows = np.stack([src[g * gs + i * rs: g * gs + i * rs + L] for i in range(k)])
        want = oracle.encode(rows, r)
        for j in range(r):
            off = g * rgs + j * rrs
            assert (rep[off: off + L] == want[j]).all(), (g, j)
            t = rep[off + L: off + tail]
            assert (t == (0 if fits and bs_shape else 0xA5)).all(), (g, j)
            if j + 1 < r:
                assert (rep[off + tail: off + rrs] == 0xA5).all()
        assert (rep[g * rgs + (r - 1) * rrs + tail: (g + 1) * rgs] == 0xA5).all()


@pytest.mark.parametrize("k,r,L,G", CASES)
@pytest.mark.parametrize("V", ["1", "2", "perm", "nofft"])
def test_encode_matches_oracle(qf, oracle, gpu_ctx, k, r, L, G, V, monkeypatch):
    # V=1/2: default dispatch (bit-sliced kernel where one exists);
    # "perm": force the general v_perm kernel
    if V == "perm":
        qf.set_default_options(bitsliced=0)
    elif V == "nofft":   # bit-sliced with one coefficient block per repair
        qf.set_default_options(fft_kernels=0)
    else:
        qf.set_default_options(encode_v=int(V))
    rng = np.random.default_rng(k * 1000 + r * 10 + L)
    rs = _r16(L) + (16 if k % 2 else 0)
    gs = k * rs + 32
    rrs = _r16(L) + 16
    rgs = r * rrs + 48
    src = rng.integers(0, 256, G * gs, dtype=np.uint8)
    rep = run_encode(qf, src, k, r, L, G, rs, gs, rrs, rgs)
    for g in range(G):
        rows = np.stack([src[g * gs + i * rs: g * gs + i * rs + L] for i in range(k)])
        want = oracle.encode(rows, r)
        for j in range(r):
            off = g * rgs + j * rrs
            assert (rep[off: off + L] == want[j]).all(), (g, j)
            assert (rep[off + L: off + rrs] == 0xA5).all(), "bytes past L written"
        assert (rep[g * rgs + r * rrs: (g + 1) * rgs] == 0xA5).all()


def test_encode_custom_coefficients(qf, oracle, gpu_ctx):
    rng = np.random.default_rng(5)
    k, r, L, G = 20, 9, 200, 6
    coeff = rng.integers(0, 256, (r, k), dtype=np.uint8)
    coeff[0, :] = 0
    coeff[1, 3] = 1
    rs = _r16(L)
    src = rng.integers(0, 256, G * k * rs, dtype=np.uint8)
    rep = run_encode(qf, src, k, r, L, G, rs, k * rs, rs, r * rs, coeff=coeff.tobytes())
    for g in range(G):
        rows = src[g * k * rs:(g + 1) * k * rs].reshape(k, rs)[:, :L]
        want = oracle.encode(rows, r, coeff)
        got = rep[g * r * rs:(g + 1) * r * rs].reshape(r, rs)[:, :L]
        assert (got == want).all()


def test_encode_golden_pattern_hashes(qf, gpu_ctx):
    for k in (16, 64):
        L = 1200
        i = np.arange(k)[:, None]
        t = np.arange(L)[None, :]
        src = ((7 * i + 13 * t + 1) & 255).astype(np.uint8).reshape(-1)
        rep = run_encode(qf, src, k, 16, L, 1, L, k * L, L, 16 * L)
        h = hashlib.sha256(rep[: 16 * L].tobytes()).hexdigest()[:32]
        assert h == GOLDEN["encode"][f"k{k}_r16_L1200_pattern"]["rep_sha"]


def test_encode_sliding_window_layout(qf, oracle, gpu_ctx):
    # adaptive.rs:519-562: after every source packet, n-k repairs over the
    # last k packets -> overlapping generations (gen stride = row stride).
    rng = np.random.default_rng(9)
    k, r, L, P = 16, 3, 96, 40
    rs = _r16(L)
    stream = rng.integers(0, 256, P * rs, dtype=np.uint8)
    G = P - k + 1
    rep = run_encode(qf, stream, k, r, L, G, rs, rs, rs, r * rs)
    for p in range(G):
        rows = stream[p * rs:(p + k) * rs].reshape(k, rs)[:, :L]
        want = oracle.encode(rows, r)
        got = rep[p * r * rs:(p + 1) * r * rs].reshape(r, rs)[:, :L]
        assert (got == want).all(), p


def test_encode_errors(qf, gpu_ctx):
    import torch

    buf = torch.zeros(1 << 16, dtype=torch.uint8, device="cuda")
    with pytest.raises(qf.QfError) as e:  # Cauchy undefined: k + r > 256
        qf.encode_batch(buf, buf, 250, 10, 16, src_row_stride=16, src_gen_stride=4000,
                        rep_row_stride=16, rep_gen_stride=160, G=1)
    assert e.value.status == -2
    with pytest.raises(qf.QfError):  # misaligned stride
        qf.encode_batch(buf, buf, 4, 2, 16, src_row_stride=17, src_gen_stride=68,
                        rep_row_stride=16, rep_gen_stride=32, G=1)


def test_gf_mul_slice_exhaustive_matches_table(qf, oracle, gpu_ctx):
    # tests/fec.rs:262-307 bitsliced_mul_matches_table / *_kernel_matches_table:
    # the device multiply equals gf_mul_table for all 65,536 pairs.
    a = np.repeat(np.arange(256, dtype=np.uint8), 256)
    b = np.tile(np.arange(256, dtype=np.uint8), 256)
    got = np.frombuffer(qf.gf_mul_slice(a.tobytes(), b.tobytes()), np.uint8).reshape(256, 256)
    assert (got == oracle.mul_table_full()).all()
    # benches/gf_mul_slice_bench.rs inputs (1024 bytes, a=i, b=255-i) and a ragged length
    a = (np.arange(1029) & 255).astype(np.uint8)
    b = (255 - np.arange(1029)).astype(np.uint8)
    got = np.frombuffer(qf.gf_mul_slice(a.tobytes(), b.tobytes()), np.uint8)
    assert all(int(got[i]) == oracle.mul(int(a[i]), int(b[i])) for i in range(1029))


BS_SHAPES = [(64, 16), (64, 10), (32, 16), (16, 16), (16, 1), (32, 5), (48, 8), (96, 15), (128, 20), (160, 48),
             (196, 59)]


@pytest.mark.parametrize("k,r", BS_SHAPES)
def test_bit_sliced_partial_last_unit_random_lengths(qf, oracle, gpu_ctx, k, r):
    """Every generated encode kernel with the zero tail at random L (mostly
    L % 16 != 0): bytes < L bit-exact, [L, round_up(L, 128)) zero, nothing
    beyond; the source rows' padding is random and must not leak."""
    rng = np.random.default_rng(1000 * k + r)
    for trial in range(3):
        L = int(rng.integers(32, 1500))
        if trial == 0:
            L |= 1                               # odd length
        G = int(rng.integers(1, 6))
        rs = _r16(L) + 16 * int(rng.integers(0, 2))
        gs = k * rs
        tail = (L + 127) // 128 * 128
        rrs = tail + 16 * int(rng.integers(0, 3))
        rgs = r * rrs
        src = rng.integers(0, 256, G * gs, dtype=np.uint8)
        rep = run_encode(qf, src, k, r, L, G, rs, gs, rrs, rgs, zero_tail=True)
        for g in range(G):
            rows = np.stack([src[g * gs + i * rs: g * gs + i * rs + L] for i in range(k)])
            want = oracle.encode(rows, r)
            for j in range(r):
                off = g * rgs + j * rrs
                assert (rep[off: off + L] == want[j]).all(), (L, g, j)
                assert (rep[off + L: off + tail] == 0).all(), (L, g, j)
                assert (rep[off + tail: off + rrs] == 0xA5).all(), (L, g, j)


@pytest.mark.parametrize("k,r", [(128, 20), (128, 39), (160, 48), (196, 59)])
def test_c5_passes_large_batch(qf, oracle, gpu_ctx, k, r):
    """C5 codes at jumbo rows with more items than CUs (the multi-item
    kernels, not the row-split 'f' ones): one launch per pass, every pass in
    one dispatch (QF_ENCODE_MERGED) and the additive-FFT coset passes
    (lch_fft.hybrid_plan) give the same repairs, block and sliding layouts;
    generations of the block batch against the oracle."""
    import torch

    L, RS = 9000, 9008
    drs = 9088
    G = 72                       # 72 x 568 units / 128 = 320 items
    gen = torch.Generator(device="cuda").manual_seed(k + r)
    src = torch.randint(0, 256, ((G + 1) * k * RS,), dtype=torch.uint8, device="cuda", generator=gen)
    out = {}
    for merged in (0, 1):
        for fft in (0, 1):
            qf.set_default_options(encode_merged=merged, fft_kernels=fft)
            for mode, gs in (("block", k * RS), ("sliding", RS)):
                rep = torch.full((G * r * drs,), 0xA5, dtype=torch.uint8, device="cuda")
                qf.encode_batch(src, rep, k, r, L, src_row_stride=RS, src_gen_stride=gs, rep_row_stride=drs,
                                rep_gen_stride=r * drs, G=G, zero_tail=True, ctx=gpu_ctx)
                gpu_ctx.sync()
                out[(merged, fft, mode)] = rep.view(G, r, drs)
    base = out[(0, 0, "block")].cpu().numpy()
    s = src.cpu().numpy()
    for key, rep in out.items():
        if not torch.equal(rep, out[(0, 0, key[2])]):
            d = np.argwhere(rep.cpu().numpy() != out[(0, 0, key[2])].cpu().numpy())
            g = int(d[0, 0])
            msg = f"{key}: {len(d)} bytes differ, gens {sorted(set(d[:, 0].tolist()))[:10]}, " \
                  f"rows {sorted(set(d[:, 1].tolist()))[:20]}, bytes {d[:3, 2].tolist()}"
            if key[2] == "block":
                w = oracle.encode(s[g * k * RS:(g + 1) * k * RS].reshape(k, RS)[:, :L], r)
                msg += f"; gen {g}: variant == oracle {bool((rep[g, :, :L].cpu().numpy() == w).all())}, " \
                       f"base == oracle {bool((base[g, :, :L] == w).all())}"
            raise AssertionError(msg)
    assert (base[:, :, L:] == 0).all()
    for g in (0, 37, G - 1):
        rows = s[g * k * RS:(g + 1) * k * RS].reshape(k, RS)[:, :L]
        assert (base[g, :, :L] == oracle.encode(rows, r)).all(), g
    sl = out[(0, 0, "sliding")].cpu().numpy()
    for g in (1, G - 1):
        rows = s[g * RS:(g + k) * RS].reshape(k, RS)[:, :L]
        assert (sl[g, :, :L] == oracle.encode(rows, r)).all(), g


def test_default_context_orders_with_torch_default_stream(qf, oracle, gpu_ctx):
    """fec.Context() on torch's default stream binds the library to the null
    stream (QF_STREAM_NULL): an encode enqueued right after torch work on that
    stream, with no synchronize in between, sees its results, and torch work
    enqueued after the encode sees the repairs."""
    import torch

    k, r, L, G = 64, 16, 1200, 4096          # large enough that an unordered read races
    assert torch.cuda.default_stream().cuda_stream == 0
    for trial in range(3):
        gen = torch.Generator(device="cuda").manual_seed(100 + trial)
        src = torch.empty(G * k * L, dtype=torch.uint8, device="cuda")
        src.copy_(torch.randint(0, 256, src.shape, dtype=torch.uint8, device="cuda", generator=gen))
        rep = torch.full((G * r * L,), 0xA5, dtype=torch.uint8, device="cuda")
        qf.encode_batch(src, rep, k, r, L, src_row_stride=L, src_gen_stride=k * L, rep_row_stride=L,
                        rep_gen_stride=r * L, G=G, ctx=gpu_ctx)
        folded = rep.view(G, r * L).to(torch.int64).sum(dim=1)    # torch, after the encode, same stream
        s = src.cpu().numpy()
        for g in (0, G // 2, G - 1):
            want = oracle.encode(s[g * k * L:(g + 1) * k * L].reshape(k, L), r)
            assert (rep[g * r * L:(g + 1) * r * L].cpu().numpy().reshape(r, L) == want).all(), (trial, g)
            assert int(folded[g]) == int(want.astype(np.int64).sum()), (trial, g)


def test_gf_mul_slice_large_table_kernel(qf, oracle, gpu_ctx):
    """Slices from 16 MiB use the 64 KiB product-table kernel: every byte
    (and the n % 16 tail) equals gf_mul_table (gf_tables.rs:47-57)."""
    import torch

    from quicfuscate_amd import _lib as L

    n = (16 << 20) + 7
    a = torch.randint(0, 256, (n + 9,), dtype=torch.uint8, device="cuda")[:n]
    b = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda")
    out = torch.empty(n + 16, dtype=torch.uint8, device="cuda").fill_(0xA5)
    torch.cuda.synchronize()
    ctx = qf.default_context()
    L.check(L._lib().qf_gf256_mul_slice_dev(ctx.handle, a.data_ptr(), b.data_ptr(), out.data_ptr(), n), "slice")
    ctx.sync()
    tab = torch.from_numpy(oracle.mul_table_full().reshape(-1)).cuda()
    want = tab[a.long() * 256 + b.long()]
    assert torch.equal(out[:n], want)
    assert (out[n:] == 0xA5).all()


@pytest.mark.parametrize("k,r,L,G", CASES + [(128, 39, 1024, 1), (64, 10, 1024, 1), (16, 1, 1024, 1),
                                             (196, 59, 9000, 1), (64, 16, 1200, 700)])
def test_encode_small_batch_kernel(qf, oracle, gpu_ctx, k, r, L, G, monkeypatch):
    """k_encode_small (lanes over generation x repair x unit; the per-packet
    send path's kernel) is bit-exact against the oracle on every case,
    including odd k (zero second coefficient), partial last units and
    k + r = 256."""
    qf.set_default_options(encode_small=1)
    rng = np.random.default_rng(k * 3 + r + L + G)
    rs = _r16(L) + 16
    gs = k * rs + 32
    src = rng.integers(0, 256, G * gs, dtype=np.uint8)
    rrs = _r16(L) + 32
    rgs = r * rrs + 16
    rep = run_encode(qf, src, k, r, L, G, rs, gs, rrs, rgs)
    for g in range(G):
        want = oracle.encode(np.stack([src[g * gs + i * rs: g * gs + i * rs + L] for i in range(k)]), r)
        for j in range(r):
            assert (rep[g * rgs + j * rrs: g * rgs + j * rrs + L] == want[j]).all(), (g, j)
            assert (rep[g * rgs + j * rrs + L: g * rgs + (j + 1) * rrs] == 0xA5).all(), (g, j)  # nothing past L


@pytest.mark.parametrize("k,r,L", [(196, 59, 2001), (160, 48, 2047), (128, 39, 4099)])
def test_c5_shared_row_encode_odd_lengths(qf, oracle, gpu_ctx, k, r, L):
    """The merged passes whose waves share their row work through LDS
    (kernels qf_cauchy_bsmx*, a producer-only wave at 3 passes) at odd row
    lengths and more items than CUs: repairs bit-exact against the oracle on
    a sample of generations, the zero tail written, nothing beyond it."""
    import torch

    rs = _r16(L)
    tail = (L + 127) // 128 * 128
    rrs = tail + 64
    items_per_gen = tail // 16 // 128 or 1
    G = 300 // items_per_gen + 8
    gs, rgs = k * rs, r * rrs
    gen = torch.Generator(device="cuda").manual_seed(k * L)
    src = torch.randint(0, 256, (G * gs,), dtype=torch.uint8, device="cuda", generator=gen)
    rep = torch.full((G * rgs,), 0xA5, dtype=torch.uint8, device="cuda")
    gpu_ctx.profile(True)
    qf.encode_batch(src, rep, k, r, L, src_row_stride=rs, src_gen_stride=gs, rep_row_stride=rrs,
                    rep_gen_stride=rgs, G=G, zero_tail=True, ctx=gpu_ctx)
    gpu_ctx.sync()
    names = set(gpu_ctx.kernel_times())
    gpu_ctx.profile(False)
    assert any(n.startswith("qf_cauchy_bsmx") for n in names), names
    s, out = src.cpu().numpy(), rep.cpu().numpy()
    for g in (0, 1, G // 2, G - 1):
        rows = s[g * gs: (g + 1) * gs].reshape(k, rs)[:, :L]
        want = oracle.encode(rows, r)
        for j in range(r):
            off = g * rgs + j * rrs
            assert (out[off: off + L] == want[j]).all(), (g, j)
            assert (out[off + L: off + tail] == 0).all(), (g, j)
            assert (out[off + tail: off + rrs] == 0xA5).all(), (g, j)


@pytest.mark.parametrize("sliding", [1, 0])
@pytest.mark.parametrize("k,r,L", [(32, 5, 9000), (48, 8, 9000), (16, 1, 1200), (48, 8, 1200), (32, 5, 1201),
                                   (64, 10, 9000), (96, 15, 9000), (128, 20, 9000), (64, 10, 1201)])
def test_encode_sliding_kernels(qf, oracle, gpu_ctx, k, r, L, sliding):
    """Overlapping generations (adaptive.rs:519-562: a window per source
    packet, generation stride = row stride) through the shapes' sliding-window
    kernels (QF_OPT_SLIDING_KERNELS = 1: cached row loads, (48, 8) as the
    hybrid FFT pass) or the block kernels (0): every checked window equals the
    oracle's encode of its k rows, and the batch equals the block layout's
    encode of the same windows."""
    import torch

    qf.set_default_options(sliding_kernels=sliding)
    RS = (L + 15) // 16 * 16 + 16
    drs = (L + 127) // 128 * 128 + 128
    G = 300
    gen = torch.Generator(device="cuda").manual_seed(k * 7 + L)
    src = torch.randint(0, 256, ((G + k - 1) * RS,), dtype=torch.uint8, device="cuda", generator=gen)
    rep = torch.full((G * r * drs,), 0xA5, dtype=torch.uint8, device="cuda")
    qf.encode_batch(src, rep, k, r, L, src_row_stride=RS, src_gen_stride=RS, rep_row_stride=drs,
                    rep_gen_stride=r * drs, G=G, zero_tail=True, ctx=gpu_ctx)
    wins = [0, 1, 77, G - 1]
    blk = torch.stack([src.view(-1, RS)[g:g + k] for g in wins]).reshape(-1)
    rb = torch.full((len(wins) * r * drs,), 0xA5, dtype=torch.uint8, device="cuda")   # same fill: bytes past the tail untouched
    qf.encode_batch(blk, rb, k, r, L, src_row_stride=RS, src_gen_stride=k * RS, rep_row_stride=drs,
                    rep_gen_stride=r * drs, G=len(wins), zero_tail=True, ctx=gpu_ctx)
    gpu_ctx.sync()
    got = rep.view(G, r, drs).cpu().numpy()
    blk_rep = rb.view(len(wins), r, drs).cpu().numpy()
    s = src.cpu().numpy()
    for n, g in enumerate(wins):
        rows = s[g * RS:(g + k) * RS].reshape(k, RS)[:, :L]
        want = oracle.encode(rows, r)
        ok_s, ok_b = bool((got[g, :, :L] == want).all()), bool((blk_rep[n, :, :L] == want).all())
        assert ok_s and ok_b, (g, "sliding batch == oracle", ok_s, "block batch == oracle", ok_b)
    assert (got[wins] == blk_rep).all()   # tails and untouched bytes too
