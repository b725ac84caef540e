"""The GF(2^8) decoder for k > 256 -- the Wiedemann strategy Decoder::new
selects there (decoder.rs:659-665, 794-975; csrc/qf_wiedemann.hip) -- against
the Wiedemann oracle (oracle/qf_oracle_wiedemann.c) bit-exact, and by round
trip (recovered rows == the original sources) at sizes the oracle cannot
finish in seconds.

Repair rows carry explicit random coefficients: the reference's Encoder
cannot make repairs for k > 256 (its u8 Cauchy rows hit gf_inv(0)),
so a k > 256 decoder only ever sees coefficient blocks supplied by the caller,
which Decoder::add_packet takes as they come (decoder.rs:693-696)."""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _feed(qf, dec, k, src, lost, coef, order="sources_first", ids=None):
    """Sources (not lost) then repairs j = 0.. with coefficient rows coef[j]."""
    r = coef.shape[0]
    L = src.shape[1]
    from tests import oracle_py as oracle

    rep = oracle.encode(src, r, coef)
    pk = []
    for i in range(k):
        if i in lost:
            continue
        pid = i if ids is None else ids[i]
        pk.append(qf.Packet(pid, bytearray(src[i].tobytes()), L, True))
    reps = [qf.Packet(10_000 + j, bytearray(rep[j].tobytes()), L, False, bytes(coef[j]), k) for j in range(r)]
    seq = pk + reps if order == "sources_first" else reps + pk
    res = [dec.add_packet(p) for p in seq]
    return res, rep


def _oracle_rows(k, src, lost, coef, rep):
    idx = [i for i in range(k) if i not in lost] + [k + j for j in range(coef.shape[0])]
    rows = np.concatenate([src[[i for i in idx if i < k]], rep])
    rc = np.zeros((len(idx), k), np.uint8)
    rc[len(idx) - coef.shape[0]:] = coef
    return idx, rows, rc


def test_strategy_follows_k(qf, gpu_ctx):
    """decoder.rs:660-664: k > 256 -> Wiedemann."""
    assert qf.Decoder(256, max_len=16).strategy == "GaussianElimination"
    assert qf.Decoder(257, max_len=16).strategy == "Wiedemann"
    assert qf.Decoder(4096, max_len=16).strategy == "Wiedemann"
    with pytest.raises(qf.QfError):
        qf.Decoder(4097, max_len=16)


def test_reference_wiedemann_path_decodes(qf, oracle, gpu_ctx):
    """src/fec/mod.rs:142-176 (and adaptive.rs:694-728): k = 260, n = 264,
    make_packet(i, i % 256) payloads in a 64-byte pool block, packets 0 and 5
    never added, all four repairs added -> decoded, out[i].data[0] == i % 256."""
    k, n = 260, 264
    pool = qf.MemoryPool(600, 64)
    src = np.zeros((k, 8), np.uint8)
    src[:] = (np.arange(k) % 256)[:, None]
    coef = np.random.default_rng(260).integers(1, 256, (n - k, k), dtype=np.uint8)
    dec = qf.Decoder(k, pool)
    assert dec.strategy == "Wiedemann"
    res, rep = _feed(qf, dec, k, src, {0, 5}, coef)
    assert dec.is_decoded and res[-1]
    out = dec.get_decoded_packets()
    assert len(out) == k
    for i in range(k):
        assert out[i].data[0] == i % 256
        assert out[i].payload() == src[i].tobytes()
    assert [p.id for p in out] == list(range(k))
    # the oracle takes the same first k rows
    idx, rows, rc = _oracle_rows(k, src, {0, 5}, coef, rep)
    s, want, mask, _ = oracle.wiedemann(k, idx, rows, rc)
    assert s == oracle.OK and (want == src).all()


@pytest.mark.parametrize("k,e,L,extra", [
    (257, 1, 1200, 0), (300, 7, 1200, 2), (512, 13, 1200, 3), (700, 32, 100, 0), (4096, 3, 64, 1),
    (333, 5, 1, 0), (400, 9, 47, 1), (1000, 2, 9000, 0),
    # e >= 64: baby-step / giant-step Krylov sequence
    (300, 64, 40, 1), (320, 97, 33, 0),
])
def test_wiedemann_vs_oracle(qf, oracle, gpu_ctx, k, e, L, extra):
    rng = np.random.default_rng(k * 31 + e)
    src = rng.integers(0, 256, (k, L), dtype=np.uint8)
    lost = set(rng.choice(k, e, replace=False).tolist())
    coef = rng.integers(0, 256, (e + extra, k), dtype=np.uint8)
    dec = qf.Decoder(k, max_len=max(L, 16))
    res, rep = _feed(qf, dec, k, src, lost, coef)
    idx, rows, rc = _oracle_rows(k, src, lost, coef, rep)
    s, want, mask, _ = oracle.wiedemann(k, idx, rows, rc)
    assert s == oracle.OK
    assert dec.is_decoded == (s == oracle.OK)
    out = dec.get_decoded_packets()
    got = np.stack([np.frombuffer(p.payload(), np.uint8) for p in out])
    assert got.shape == want.shape
    assert (got == want).all() and (got == src).all()
    assert [p.id for p in out] == list(range(k))


@pytest.mark.parametrize("k,e,L", [(600, 200, 48), (2048, 64, 1200), (4096, 40, 1500), (300, 299, 32)])
def test_wiedemann_round_trip_large(qf, gpu_ctx, k, e, L):
    """Sizes the oracle does not finish in seconds: recovered == sources."""
    rng = np.random.default_rng(k + e)
    src = rng.integers(0, 256, (k, L), dtype=np.uint8)
    lost = set(rng.choice(k, e, replace=False).tolist())
    coef = rng.integers(0, 256, (e, k), dtype=np.uint8)
    dec = qf.Decoder(k, max_len=L)
    _feed(qf, dec, k, src, lost, coef, order="repairs_first")
    assert dec.is_decoded
    out = dec.get_decoded_packets()
    got = np.stack([np.frombuffer(p.payload(), np.uint8) for p in out])
    assert (got == src).all()


def test_wiedemann_singular_stays_undecoded(qf, oracle, gpu_ctx):
    """Two equal repair rows: rank k - 1, so the decoder stays undecoded
    (decoder.rs:852-854 returns false) and the oracle reports ERANK."""
    k, L = 300, 64
    rng = np.random.default_rng(1)
    src = rng.integers(0, 256, (k, L), dtype=np.uint8)
    lost = {3, 100, 299}
    coef = rng.integers(1, 256, (3, k), dtype=np.uint8)
    coef[2] = coef[1]
    dec = qf.Decoder(k, max_len=L)
    res, rep = _feed(qf, dec, k, src, lost, coef)
    assert not any(res) and not dec.is_decoded
    assert dec.get_decoded_packets() == []
    idx, rows, rc = _oracle_rows(k, src, lost, coef, rep)
    assert oracle.wiedemann(k, idx, rows, rc)[0] == oracle.ERANK
    # a zero coefficient row on an erased column block: singular too
    coef2 = coef.copy()
    coef2[2] = 0
    dec = qf.Decoder(k, max_len=L)
    res, _ = _feed(qf, dec, k, src, lost, coef2)
    assert not dec.is_decoded


def test_wiedemann_no_loss_duplicates_and_short(qf, gpu_ctx):
    k, L = 290, 20
    rng = np.random.default_rng(2)
    src = rng.integers(0, 256, (k, L), dtype=np.uint8)
    # no loss: decodes on the k-th systematic row, no repair needed
    dec = qf.Decoder(k, max_len=L)
    res, _ = _feed(qf, dec, k, src, set(), np.zeros((0, k), np.uint8))
    assert res[-1] and dec.is_decoded
    got = np.stack([np.frombuffer(p.payload(), np.uint8) for p in dec.get_decoded_packets()])
    assert (got == src).all()
    # duplicates of received sources are dropped (decoder.rs:687-691); one row short stays undecoded
    dec = qf.Decoder(k, max_len=L)
    for i in (1, 2, 3):
        dec.add_packet(qf.Packet(i, bytearray(src[i].tobytes()), L, True))
    coef = rng.integers(1, 256, (4, k), dtype=np.uint8)
    res, _ = _feed(qf, dec, k, src, {10, 20, 30, 40}, coef[:3])
    assert not dec.is_decoded
    # 286 sources + 3 repairs: one row short.  One more repair (no sources
    # re-sent) makes k rows
    res, _ = _feed(qf, dec, k, src, set(range(k)), coef[3:])
    assert dec.is_decoded
    got = np.stack([np.frombuffer(p.payload(), np.uint8) for p in dec.get_decoded_packets()])
    assert (got == src).all()


def test_received_ids_kept(qf, gpu_ctx):
    """A received systematic packet keeps its own id, a recovered one gets i
    (decoder.rs:688, 889-905)."""
    k, L = 270, 16
    rng = np.random.default_rng(3)
    src = rng.integers(0, 256, (k, L), dtype=np.uint8)
    ids = [k * 20 + i for i in range(k)]   # id % k == i, id != i
    assert all(x % k == i for i, x in enumerate(ids))
    lost = {0, 269}
    coef = rng.integers(1, 256, (2, k), dtype=np.uint8)
    dec = qf.Decoder(k, max_len=L)
    _feed(qf, dec, k, src, lost, coef, ids=ids)
    assert dec.is_decoded
    out = dec.get_decoded_packets()
    assert [p.id for p in out] == [i if i in lost else ids[i] for i in range(k)]


@pytest.mark.parametrize("proj", [0, 1])
@pytest.mark.parametrize("k,lost_n", [(300, 300), (400, 40)])
def test_wiedemann_exact_fallback(qf, oracle, gpu_ctx, qf_opts, k, lost_n, proj):
    """A matrix crafted against the reference's init vectors: M on the erased
    block is diag(c), c = 7 on positions {0, 1, 16, 17} of E and 11 elsewhere
    -- the init vectors b < 8 XOR to zero over those positions, so none of
    them sees the eigenvalue 7.  With the reference's vectors only
    (QF_OPT_WIEDEMANN_PROJ 0) no projection verifies and exact elimination on
    the host decides (solve_attempts 9); with the default random projections
    after the first (a sender must not be able to force the host
    fallback) a projection verifies.  M is nonsingular, so the generation
    decodes either way, as in the oracle; the received columns carry random
    coefficients."""
    qf_opts(wiedemann_proj=proj)
    rng = np.random.default_rng(k)
    L = 40
    src = rng.integers(0, 256, (k, L), dtype=np.uint8)
    E = sorted(rng.choice(k, lost_n, replace=False).tolist()) if lost_n < k else list(range(k))
    lost = set(E)
    coef = np.zeros((lost_n, k), np.uint8)
    recv = [i for i in range(k) if i not in lost]
    if recv:
        coef[:, recv] = rng.integers(0, 256, (lost_n, len(recv)), dtype=np.uint8)
    for p, col in enumerate(E):
        coef[p, col] = 7 if p in (0, 1, 16, 17) else 11
    dec = qf.Decoder(k, max_len=L)
    res, rep = _feed(qf, dec, k, src, lost, coef)
    assert dec.is_decoded and res[-1]
    assert dec.solve_attempts == 9 if proj == 0 else 2 <= dec.solve_attempts <= 8
    got = np.stack([np.frombuffer(p.payload(), np.uint8) for p in dec.get_decoded_packets()])
    assert (got == src).all()
    idx, rows, rc = _oracle_rows(k, src, lost, coef, rep)
    s, want, _, _ = oracle.wiedemann(k, idx, rows, rc)
    assert s == oracle.OK and (want == got).all()
    # a zero on M's diagonal: singular, stays undecoded
    coef[3, E[3]] = 0
    dec = qf.Decoder(k, max_len=L)
    _feed(qf, dec, k, src, lost, coef)
    assert not dec.is_decoded


def test_wiedemann_exact_fallback_cost_pinned(qf, gpu_ctx, qf_opts):
    """The host fallback's cost at the largest erased block a test can afford
    to force (QF_OPT_WIEDEMANN_PROJ 0, e = k = 1,024, the crafted diagonal of
    test_wiedemann_exact_fallback): O(e^3 / 16) pshufb steps, well under a
    second here; with the default random projections the same input never
    reaches it (and e = 4,096 would cost about 64x more)."""
    import time

    k = 1024
    L = 16
    rng = np.random.default_rng(7)
    src = rng.integers(0, 256, (k, L), dtype=np.uint8)
    coef = np.zeros((k, k), np.uint8)
    for p in range(k):
        coef[p, p] = 7 if p in (0, 1, 16, 17) else 11
    for proj, want in ((0, 9), (1, None)):
        qf_opts(wiedemann_proj=proj)
        dec = qf.Decoder(k, max_len=L)
        t0 = time.perf_counter()
        _feed(qf, dec, k, src, set(range(k)), coef)
        dt = time.perf_counter() - t0
        assert dec.is_decoded
        got = np.stack([np.frombuffer(p.payload(), np.uint8) for p in dec.get_decoded_packets()])
        assert (got == src).all()
        if want is None:
            assert dec.solve_attempts <= 8
        else:
            assert dec.solve_attempts == want
            assert dt < 10.0, f"exact fallback at e = {k}: {dt:.2f} s"
