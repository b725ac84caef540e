"""Heterogeneous batches (qf_encode_batch_desc / qf_decode_batch_desc,
SURVEY 8(b) qf_gen_desc): one call over generations whose (k, r, L) differ
per generation -- BASELINE C5's ASW-RLNC-X mix, k drawn per generation from
the Normal / Medium windows with r = ceil(k * ratio) - k (adaptive.rs:124-153)
-- placed at shuffled, gapped offsets.  Every generation's repairs and
recovered rows are checked against the oracle (decoder.rs:172-275, 678-783)."""

import numpy as np
import pytest

from quicfuscate_amd import _lib as L

pytestmark = pytest.mark.gpu

# (k, r): Normal ratio 1.15 for k <= 128, Medium 1.30 above
C5 = [(32, 5), (48, 8), (64, 10), (96, 15), (128, 20), (160, 48), (196, 59)]


def _r16(x):
    return (x + 15) // 16 * 16


def _layout(rng, sizes, gap=48):
    """Byte offsets of blocks of the given sizes, shuffled order, gaps between."""
    order = rng.permutation(len(sizes))
    offs = [0] * len(sizes)
    pos = 0
    for i in order:
        offs[i] = pos
        pos = _r16(pos + sizes[i] + int(rng.integers(0, 4)) * gap)
    return offs, pos + 256


def _plan(rng, n_gen, Ls):
    gens = []
    for q in range(n_gen):
        k, r = C5[q % len(C5)] if q < len(C5) else C5[int(rng.integers(0, len(C5)))]
        gens.append((k, r, int(Ls[q % len(Ls)])))
    return gens


@pytest.mark.parametrize("Ls,zero_tail", [((1200, 336, 64), False), ((1200, 9000), True)])
def test_encode_desc_mixed_windows(qf, oracle, gpu_ctx, Ls, zero_tail):
    import torch

    rng = np.random.default_rng(len(Ls) * 7 + zero_tail)
    gens = _plan(rng, 16 if zero_tail else 24, Ls)
    Lp = lambda Lb: 16 * ((_r16(Lb) // 16 + 7) // 8 * 8) if zero_tail else _r16(Lb)  # noqa: E731
    src_off, src_bytes = _layout(rng, [k * _r16(Lb) for k, r, Lb in gens])
    rep_off, rep_bytes = _layout(rng, [r * Lp(Lb) for k, r, Lb in gens])
    src_np = rng.integers(0, 256, src_bytes, dtype=np.uint8)
    src = torch.from_numpy(src_np).cuda()
    rep = torch.full((rep_bytes,), 0xEE, dtype=torch.uint8, device="cuda")
    descs = [dict(k=k, r=r, L=Lb, flags=1 if zero_tail else 0, src_offset=src_off[q], src_row_stride=_r16(Lb),
                  rep_offset=rep_off[q], rep_row_stride=Lp(Lb)) for q, (k, r, Lb) in enumerate(gens)]
    qf.encode_batch_desc(src, rep, descs)
    qf.default_context().sync()
    out = rep.cpu().numpy()
    for q, (k, r, Lb) in enumerate(gens):
        so, ro, rs = src_off[q], rep_off[q], _r16(Lb)
        rows = src_np[so: so + k * rs].reshape(k, rs)[:, :Lb]
        want = oracle.encode(rows, r)
        got = out[ro: ro + r * Lp(Lb)].reshape(r, Lp(Lb))
        assert (got[:, :Lb] == want).all(), (q, k, r, Lb)
        tail = got[:, Lb:]
        if zero_tail:   # the library MAY zero [L, Lp) (bit-sliced path) or leave it (small-batch path)
            assert all((t == 0).all() or (t == 0xEE).all() for t in tail), (q, k, r, Lb)
        else:
            assert (tail == 0xEE).all()


def test_encode_desc_errors(qf, gpu_ctx):
    import torch

    buf = torch.zeros(1 << 16, dtype=torch.uint8, device="cuda")
    with pytest.raises(qf.QfError) as e:   # k + r > 256: the reference panics in gf_inv(0)
        qf.encode_batch_desc(buf, buf, [dict(k=200, r=60, L=64, src_row_stride=64, rep_row_stride=64)])
    assert e.value.status == L.QF_ERANGE
    with pytest.raises(qf.QfError) as e:   # offsets must be 16-byte aligned
        qf.encode_batch_desc(buf, buf, [dict(k=4, r=2, L=64, src_offset=8, src_row_stride=64, rep_row_stride=64)])
    assert e.value.status == L.QF_EINVAL
    qf.encode_batch_desc(buf, buf, [])     # empty batch: no-op


def test_decode_desc_mixed_windows(qf, oracle, gpu_ctx):
    import torch

    rng = np.random.default_rng(99)
    gens = _plan(rng, 21, (1200, 336, 9000, 64))
    # encode each generation (oracle), choose erasures, arrival order
    plans = []
    for q, (k, r, Lb) in enumerate(gens):
        src = rng.integers(0, 256, (k, Lb), dtype=np.uint8)
        rep = oracle.encode(src, r)
        emax = min(k, r)
        if q == 3:
            e, n_rep = 2, 1            # fewer than k rows: ENOTREADY
        elif q == 5:
            e, n_rep = 0, 0            # nothing lost
        else:
            e = int(rng.integers(1, emax + 1))
            n_rep = min(r, e + int(rng.integers(0, 3)))
        E = sorted(rng.choice(k, e, replace=False).tolist())
        J = sorted(rng.choice(r, n_rep, replace=False).tolist())
        arr = [i for i in range(k) if i not in E] + [k + j for j in J]
        arr = [arr[i] for i in rng.permutation(len(arr))]
        rows = np.stack([src[a] if a < k else rep[a - k] for a in arr])
        plans.append((src, E, arr, rows))
    rs = [_r16(Lb) for _, _, Lb in gens]
    row_off, rows_bytes = _layout(rng, [len(p[2]) * rs[q] for q, p in enumerate(plans)])
    rec_off, rec_bytes = _layout(rng, [min(k, r) * rs[q] for q, (k, r, _) in enumerate(gens)])
    ri_off, pos = [], 0
    for p in plans:
        ri_off.append(pos)
        pos += len(p[2]) + 3
    ci_off, cpos = [], 0
    for k, r, _ in gens:
        ci_off.append(cpos)
        cpos += min(k, r) + 1
    rows_np = np.zeros(rows_bytes, np.uint8)
    ri_np = np.full(pos + 1, 0x7777, np.uint16)
    for q, (src, E, arr, rows) in enumerate(plans):
        Lb = gens[q][2]
        for s, row in enumerate(rows):
            rows_np[row_off[q] + s * rs[q]: row_off[q] + s * rs[q] + Lb] = row
        ri_np[ri_off[q]: ri_off[q] + len(arr)] = arr
    t_rows = torch.from_numpy(rows_np).cuda()
    t_ri = torch.from_numpy(ri_np.view(np.int16)).cuda()
    t_rec = torch.full((rec_bytes,), 0xEE, dtype=torch.uint8, device="cuda")
    t_ci = torch.full((cpos + 1,), -1, dtype=torch.int16, device="cuda")
    t_n = torch.full((len(gens),), 999, dtype=torch.int32, device="cuda")
    t_st = torch.full((len(gens),), 999, dtype=torch.int32, device="cuda")
    descs = [dict(k=k, r=r, L=Lb, n_rows=len(plans[q][2]), rows_offset=row_off[q], row_stride=rs[q],
                  row_index_offset=ri_off[q], rec_offset=rec_off[q], rec_row_stride=rs[q],
                  rec_index_offset=ci_off[q]) for q, (k, r, Lb) in enumerate(gens)]
    qf.decode_batch_desc(t_rows, t_ri, t_rec, t_ci, t_n, t_st, descs)
    qf.default_context().sync()
    rec = t_rec.cpu().numpy()
    ci = t_ci.cpu().numpy().view(np.uint16)
    n_rec, st = t_n.cpu().numpy(), t_st.cpu().numpy()
    for q, (k, r, Lb) in enumerate(gens):
        src, E, arr, rows = plans[q]
        ost, sol, mask = oracle.decode(k, arr, rows)
        assert st[q] == ost, (q, st[q], ost)
        if ost != 0:
            continue
        # first k rows win (decoder.rs:679): a source arriving after the k-th
        # row is recovered too, so the recovered set is the oracle's, not E
        erased = [int(i) for i in np.nonzero(mask == 0)[0]]
        assert set(E) <= set(erased) and n_rec[q] == len(erased)
        assert list(ci[ci_off[q]: ci_off[q] + len(erased)]) == erased
        for m, i in enumerate(erased):
            got = rec[rec_off[q] + m * rs[q]: rec_off[q] + m * rs[q] + Lb]
            assert (got == sol[i]).all() and (got == src[i]).all(), (q, m)
