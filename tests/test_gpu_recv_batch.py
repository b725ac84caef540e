"""Multi-connection receive batches (qf_adaptive_on_receive_batch): M
connection states each receive one packet per call; their rows go up in one
copy and the generations that complete in the call decode together.  Every
connection's recovered packets and statuses equal its twin driven by
per-packet on_receive (adaptive.rs:566-599), and every recovered payload is
the sender's original (decoder.rs:678-791)."""
import numpy as np
import pytest

from quicfuscate_amd import _lib as L

pytestmark = pytest.mark.gpu


def _cfg(qf, mode, max_len=1500, normal=64, extreme=None):
    w = qf.default_windows()
    w[qf.FecMode.Normal] = normal
    if extreme:
        w[qf.FecMode.Extreme] = extreme
    return qf.FecConfig(initial_mode=mode, max_len=max_len, window_sizes=w)


def _stream(qf, cfg, rng, n_src, lens, lost, base_id):
    """The packets a sender emits for n_src sources (sliding window), with the
    source indices in `lost` dropped; returns (packets in arrival order,
    original payloads by id)."""
    snd = qf.AdaptiveFec(cfg, now=0.0)
    out, orig = [], {}
    for i in range(n_src):
        ln = int(lens[i % len(lens)])
        b = rng.integers(0, 256, ln, dtype=np.uint8).tobytes()
        orig[base_id + i] = b
        q = []
        snd.on_send(qf.Packet(base_id + i, bytearray(b), ln, True), q)
        for p in q:
            if p.is_systematic and (p.id - base_id) in lost:
                continue
            out.append(p)
    return out, orig


def _same(a, b):
    return [(p.id, p.len, p.payload()) for p in a] == [(p.id, p.len, p.payload()) for p in b]


def test_recv_batch_mixed_connections(qf, gpu_ctx):
    M = qf.FecMode
    rng = np.random.default_rng(21)
    kinds = [
        ("normal64", _cfg(qf, M.Normal), (1200,), {3, 17, 40}, 70),
        ("normal24", _cfg(qf, M.Normal, normal=24), (1200, 700), {0, 5}, 30),
        ("light", _cfg(qf, M.Light, max_len=300), (300, 64, 8), {2}, 20),
        ("light_dup", _cfg(qf, M.Light), (64,), {9}, 24),          # twice per call
        ("extreme", _cfg(qf, M.Extreme, extreme=24), (40,), {4}, 30),   # GF(2^16): per-connection path
        ("zero", _cfg(qf, M.Zero), (100,), set(), 8),
        ("strong", _cfg(qf, M.Strong), (32,), set(), 8),                # no GF(2^8) code: nothing decodes
    ]
    streams, recv, twin, origs = {}, {}, {}, {}
    for n, (name, cfg, lens, lost, n_src) in enumerate(kinds):
        pk, orig = _stream(qf, cfg, rng, n_src, lens, lost, 0)   # ids from 0: column id % k = window position
        streams[name] = pk
        origs[name] = orig
        recv[name] = qf.AdaptiveFec(cfg, now=0.0)
        twin[name] = qf.AdaptiveFec(cfg, now=0.0)
    # a repair without coefficients: QF_EINVAL for that packet only
    bad = streams["normal24"][3]
    streams["normal24"].insert(4, qf.Packet(bad.id + 500, bytearray(b"x" * 16), 16, False, None, 0))
    cursor = {name: 0 for name in streams}
    got = {name: [] for name in streams}
    rounds = 0
    while any(cursor[n] < len(streams[n]) for n in streams):
        order = [n for n in streams if cursor[n] < len(streams[n])]
        if cursor["light_dup"] + 1 < len(streams["light_dup"]):
            order.append("light_dup")
        order = [order[i] for i in rng.permutation(len(order))]
        fecs, pkts, names = [], [], []
        for n in order:
            fecs.append(recv[n])
            pkts.append(streams[n][cursor[n]])
            names.append(n)
            cursor[n] += 1
        res, st = qf.on_receive_batch(fecs, pkts)
        for n, p, r, s in zip(names, pkts, res, st):
            try:
                want = twin[n].on_receive(p)
                ws = L.QF_OK
            except qf.QfError as e:
                want, ws = [], e.status
            assert s == ws, (n, p.id, s, ws)
            assert _same(r, want), (n, p.id)
            got[n] += r
        rounds += 1
    assert rounds > 60
    for name in ("normal64", "normal24", "light", "light_dup"):
        k = recv[name].state()["k"]
        assert len(got[name]) == k, name
        for p in got[name]:
            # received systematic packets keep their id, recovered ones get i (= the
            # id here) and the generation's length L = window[0].len, zero padded
            o = origs[name][p.id]
            assert p.payload()[: len(o)] == o and not any(p.payload()[len(o):]), (name, p.id)
    assert got["strong"] == [] and got["zero"] == []


def test_recv_batch_many_generations_decode_together(qf, gpu_ctx):
    """256 connections complete their generation in the same call: one
    batched decode of 256 generations; every erased source comes back."""
    M = qf.FecMode
    rng = np.random.default_rng(5)
    cfg = _cfg(qf, M.Normal, normal=20, max_len=1200)
    conns, streams, origs = [], [], []
    for c in range(256):
        lost = set(rng.choice(20, int(rng.integers(1, 4)), replace=False).tolist())
        pk, orig = _stream(qf, cfg, rng, 20, (1200, 1024, 555), lost, 0)
        # arrival: survivors then the window's repairs; pad with the spare
        # repairs so every stream has the same length
        conns.append(qf.AdaptiveFec(cfg, now=0.0))
        streams.append(pk)
        origs.append(orig)
    n_max = max(len(s) for s in streams)
    got = [[] for _ in conns]
    for t in range(n_max):
        idx = [c for c in range(len(conns)) if t < len(streams[c])]
        res, st = qf.on_receive_batch([conns[c] for c in idx], [streams[c][t] for c in idx])
        assert st == [L.QF_OK] * len(idx)
        for c, r in zip(idx, res):
            got[c] += r
    for c in range(len(conns)):
        assert len(got[c]) == 20
        for p in got[c]:
            o = origs[c][p.id]
            assert p.payload()[: len(o)] == o and not any(p.payload()[len(o):]), (c, p.id)


def test_recv_batch_explicit_coefficients_and_second_context(qf, gpu_ctx):
    """Repairs whose coefficient vectors are not Cauchy rows of the
    generation take the per-decoder Gauss-Jordan path inside the batch, and
    a connection on another context takes the per-connection path; both equal
    their per-packet twins."""
    M = qf.FecMode
    rng = np.random.default_rng(77)
    cfg = _cfg(qf, M.Normal, normal=20, max_len=512)
    ctx2 = qf.Context(0)
    recv = [qf.AdaptiveFec(cfg, now=0.0) for _ in range(3)] + [qf.AdaptiveFec(cfg, now=0.0, ctx=ctx2)]
    twin = [qf.AdaptiveFec(cfg, now=0.0) for _ in range(4)]
    k = recv[0].state()["k"]
    streams = []
    for c in range(4):
        src = [rng.integers(0, 256, 512, dtype=np.uint8).tobytes() for _ in range(k)]
        pk = [qf.Packet(i, bytearray(src[i]), 512, True) for i in range(k) if i not in (2, 11)]
        for j in range(3):   # random (invertible with high probability) coefficient vectors
            co = rng.integers(1, 256, k, dtype=np.uint8)
            pay = rng.integers(0, 256, 512, dtype=np.uint8).tobytes()
            pk.append(qf.Packet(k + j, bytearray(pay), 512, False, bytes(co), k))
        streams.append(pk)
    for t in range(len(streams[0])):
        res, st = qf.on_receive_batch(recv, [s[t] for s in streams])
        for c in range(4):
            want = twin[c].on_receive(streams[c][t])
            assert st[c] == L.QF_OK and _same(res[c], want), (t, c)
