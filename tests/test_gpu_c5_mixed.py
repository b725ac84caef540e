"""BASELINE C5: adaptive sliding-window mixed generations,
9000-byte jumbo payloads, r = ceil(k * ratio) - k in f32 (Normal 1.15 for
k <= 128, Medium 1.30 above), block mode and sliding mode (stride 1), each
generation size its own batch call -- bit-exact against the oracle, and a
decode round trip at the maximum erasure count of every shape."""
import numpy as np
import pytest

from quicfuscate_amd import _lib as L

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _bit_sliced_encode(qf):
    # these tests pin the bit-sliced kernels (and their zero tails) at small
    # G; the small-batch kernel has its own cases (test_gpu_encode.py)
    qf.set_default_options(encode_small=0)
L_JUMBO = 9000
RS = 9008          # row stride: 16-byte multiple (C ABI), rows zero padded
REP_RS = 9088      # pool-block repair rows: round_up(9000, 128), the zero tail fits
SHAPES = [(k, int(np.ceil(np.float32(k) * np.float32(ratio))) - k)
          for k, ratio in ((32, 1.15), (48, 1.15), (64, 1.15), (96, 1.15), (128, 1.15), (160, 1.30), (196, 1.30))]


def test_c5_shapes():
    assert [r for _, r in SHAPES] == [5, 8, 10, 15, 20, 48, 59]
    assert max(k + r for k, r in SHAPES) == 255


@pytest.mark.parametrize("k,r", SHAPES)
@pytest.mark.parametrize("sliding", [False, True])
@pytest.mark.parametrize("zero_tail", [False, True])
def test_c5_encode_matches_oracle(qf, oracle, gpu_ctx, k, r, sliding, zero_tail):
    """zero_tail: pool-block repair rows (QF_ENCODE_ZERO_TAIL) run the
    bit-sliced pass kernels with the masked partial last unit; without it,
    the general kernel writes exactly L bytes."""
    import torch

    rng = np.random.default_rng(k * 7 + sliding)
    G = 3
    rs = RS
    drs = REP_RS if zero_tail else RS
    if sliding:   # one window per source packet: generation stride = row stride
        P = k + G - 1
        src = rng.integers(0, 256, P * rs, dtype=np.uint8)
        gs = rs
    else:
        src = rng.integers(0, 256, G * k * rs, dtype=np.uint8)
        gs = k * rs
    t_src = torch.from_numpy(src).cuda()
    rep = torch.full((G * r * drs,), 0xEE, dtype=torch.uint8, device="cuda")
    qf.encode_batch(t_src, rep, k, r, L_JUMBO, src_row_stride=rs, src_gen_stride=gs, rep_row_stride=drs,
                    rep_gen_stride=r * drs, G=G, zero_tail=zero_tail)
    qf.default_context().sync()
    got = rep.cpu().numpy().reshape(G, r, drs)
    for g in range(G):
        rows = src[g * gs: g * gs + k * rs].reshape(k, rs)[:, :L_JUMBO]
        assert (got[g][:, :L_JUMBO] == oracle.encode(rows, r)).all(), g
        # the library writes [L, 16 * padded units) as zeros with the flag, else nothing past L
        assert (got[g][:, L_JUMBO:] == (0 if zero_tail else 0xEE)).all(), g


@pytest.mark.parametrize("k,r", SHAPES)
def test_c5_decode_round_trip(qf, oracle, gpu_ctx, k, r):
    import torch

    rng = np.random.default_rng(k)
    G = 2
    e = min(k, r)
    src = rng.integers(0, 256, (G, k, L_JUMBO), dtype=np.uint8)
    reps = np.stack([oracle.encode(src[g], r) for g in range(G)])
    max_rows = k - e + r
    rows = np.zeros((G, max_rows, RS), np.uint8)
    ridx = np.zeros((G, max_rows), np.uint16)
    erased = []
    for g in range(G):
        E = sorted(rng.choice(k, e, replace=False).tolist())
        erased.append(E)
        arr = [i for i in range(k) if i not in E] + [k + j for j in range(r)]
        ridx[g] = arr
        rows[g, :, :L_JUMBO] = np.stack([src[g, a] if a < k else reps[g, a - k] for a in arr])
    rec = torch.empty(G * e * RS, dtype=torch.uint8, device="cuda")
    rec_index = torch.empty(G * e, dtype=torch.int16, device="cuda")
    n_rec = torch.empty(G, dtype=torch.int32, device="cuda")
    status = torch.empty(G, dtype=torch.int32, device="cuda")
    qf.decode_batch(torch.from_numpy(rows.reshape(-1)).cuda(), torch.from_numpy(ridx.view(np.int16).reshape(-1)).cuda(),
                    rec, rec_index, n_rec, status, k, r, L_JUMBO, max_rows=max_rows, row_stride=RS,
                    rows_gen_stride=max_rows * RS, rec_row_stride=RS, rec_gen_stride=e * RS, G=G)
    qf.default_context().sync()
    assert (status.cpu().numpy() == 0).all()
    assert (n_rec.cpu().numpy() == e).all()
    recv = rec.cpu().numpy().reshape(G, e, RS)[:, :, :L_JUMBO]
    idx = rec_index.cpu().numpy().view(np.uint16).reshape(G, e)
    for g in range(G):
        assert list(idx[g]) == erased[g]
        assert (recv[g] == src[g, erased[g]]).all()
