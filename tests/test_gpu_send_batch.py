"""Multi-connection send batches (qf_adaptive_on_send_batch): M connection
states each send one packet per call, the steady GF(2^8) ones through one
upload, one small-batch encode launch per (k, n) class and one download.
Every connection's output equals its twin driven by per-packet on_send
(adaptive.rs:519-562), and every GF(2^8) repair equals the oracle's encode
of that connection's window (decoder.rs:172-275)."""
import ctypes

import numpy as np
import pytest

from quicfuscate_amd import _lib as L

pytestmark = pytest.mark.gpu


def _cfg(qf, mode, max_len=1500, **kw):
    w = qf.default_windows()
    w[qf.FecMode.Normal] = kw.pop("normal_window", 64)
    return qf.FecConfig(initial_mode=mode, max_len=max_len, window_sizes=w, **kw)


def _pair(qf, cfg, codec=True):
    return qf.AdaptiveFec(cfg, now=0.0, codec=codec), qf.AdaptiveFec(cfg, now=0.0, codec=codec)


def _same(p, q):
    return (p.id, p.len, p.is_systematic, p.payload(), p.coeff_len,
            None if p.coefficients is None else bytes(p.coefficients[: p.coeff_len])) == \
           (q.id, q.len, q.is_systematic, q.payload(), q.coeff_len,
            None if q.coefficients is None else bytes(q.coefficients[: q.coeff_len]))


def _check_oracle(oracle, k, r, hist, reps):
    """reps: repairs emitted right after hist[-1] was sent (window = hist[-k:])."""
    win = hist[-k:]
    Lw = len(win[0])
    stride = max([Lw] + [len(b) for b in win])
    src = np.zeros((k, max(stride, 1)), np.uint8)
    for i, b in enumerate(win):
        src[i, : len(b)] = np.frombuffer(b, np.uint8)
    want = oracle.encode(src, r, L=Lw)
    C = oracle.cauchy(k, r)
    assert len(reps) == r
    for j, p in enumerate(reps):
        assert p.len == Lw and p.payload() == want[j, :Lw].tobytes()
        assert p.coeff_len == k and bytes(p.coefficients) == bytes(C[j])


def test_send_batch_mixed_connections(qf, oracle, gpu_ctx):
    M = qf.FecMode
    specs = [
        ("normal64", _cfg(qf, M.Normal), True, 1200),
        ("normal24", _cfg(qf, M.Normal, normal_window=24), True, 1200),
        ("light_short_stride", _cfg(qf, M.Light, max_len=300), True, 300),
        ("light_dup", _cfg(qf, M.Light), True, 64),          # appears twice per call
        ("extreme", None, True, 40),                         # GF(2^16): per-connection path
        ("zero", _cfg(qf, M.Zero), True, 100),
        ("controller", _cfg(qf, M.Normal), False, 100),
        ("fade", _cfg(qf, M.Normal, pid=qf.PidConfig(1.0, 0.0, 0.0), lambda_=0.01, burst_window=50), True, 16),
        ("strong", _cfg(qf, M.Strong), True, 32),            # QF_ERANGE: no GF(2^8) code
    ]
    w = qf.default_windows()
    w[qf.FecMode.Extreme] = 24
    specs[4] = ("extreme", qf.FecConfig(initial_mode=M.Extreme, window_sizes=w), True, 40)
    names = [s[0] for s in specs]
    pairs = {name: _pair(qf, cfg, codec) for name, cfg, codec, _ in specs}
    maxlen = {name: ml for name, _, _, ml in specs}
    pairs["fade"][0].report_loss(0, 20, now=1.0)
    pairs["fade"][1].report_loss(0, 20, now=1.0)
    assert pairs["fade"][0].is_transitioning()
    rng = np.random.default_rng(7)
    hist = {n: [] for n in names}
    next_id = {n: 1000 * i for i, n in enumerate(names)}
    n_checked = 0
    for rnd in range(72):
        order = names + ["light_dup"]
        order = [order[i] for i in rng.permutation(len(order))]
        fecs, pkts = [], []
        for n in order:
            ln = int(rng.integers(0, maxlen[n] + 1)) if rnd % 5 else maxlen[n]
            b = rng.integers(0, 256, ln, dtype=np.uint8).tobytes()
            fecs.append(pairs[n][0])
            pkts.append((n, qf.Packet(next_id[n], bytearray(b), ln, True)))
            next_id[n] += 1
        queues, st = qf.on_send_batch(fecs, [p for _, p in pkts])
        for m, (n, p) in enumerate(pkts):
            twin_out = []
            s = pairs[n][1].on_send(qf.Packet(p.id, bytearray(p.payload()), p.len, True), twin_out)
            assert st[m] == s, (rnd, n)
            assert len(queues[m]) == len(twin_out), (rnd, n)
            assert all(_same(a, b) for a, b in zip(queues[m], twin_out)), (rnd, n)
            hist[n].append(p.payload())
            sd = pairs[n][0].state()
            if n in ("normal64", "normal24", "light_short_stride", "light_dup") and len(queues[m]) > 1:
                _check_oracle(oracle, sd["k"], sd["n"] - sd["k"], hist[n], queues[m][1:])
                n_checked += 1
        assert pairs["fade"][0].state() == pairs["fade"][1].state()
    assert n_checked > 100
    assert not pairs["fade"][0].is_transitioning()


def test_send_batch_many_connections(qf, oracle, gpu_ctx):
    """384 connections in three (k, n) classes (r = 3, 1, 12: the all-repairs
    tile kernel with one and two repair chunks), full windows from the k-th call."""
    M = qf.FecMode
    w = qf.default_windows()
    w[M.Medium] = 40
    cfgs = [_cfg(qf, M.Normal, normal_window=20, max_len=1200), _cfg(qf, M.Light, max_len=1200),
            qf.FecConfig(initial_mode=M.Medium, max_len=1200, window_sizes=w)]
    fecs = [qf.AdaptiveFec(cfgs[i % 3], now=0.0) for i in range(384)]
    ks = [f.state()["k"] for f in fecs]
    rng = np.random.default_rng(11)
    hist = [[] for _ in fecs]
    for rnd in range(max(ks) + 2):
        pays = [rng.integers(0, 256, 1200 if (rnd + m) % 3 else int(rng.integers(1, 1200)), dtype=np.uint8).tobytes()
                for m in range(len(fecs))]
        queues, st = qf.on_send_batch(fecs, [qf.Packet(rnd, bytearray(b), len(b), True) for b in pays])
        assert st == [L.QF_OK] * len(fecs)
        for m, f in enumerate(fecs):
            hist[m].append(pays[m])
            k, n = f.state()["k"], f.state()["n"]
            assert queues[m][0].payload() == pays[m]
            if rnd + 1 < k:
                assert len(queues[m]) == 1
            elif m % 7 == 0 or rnd == max(ks) + 1:
                _check_oracle(oracle, k, n - k, hist[m], queues[m][1:])


def test_send_batch_argument_errors(qf, gpu_ctx):
    lib = L._lib()
    f = qf.AdaptiveFec(_cfg(qf, qf.FecMode.Light, max_len=100), now=0.0)
    conns = (ctypes.c_void_p * 2)(f.handle, f.handle)
    ids = (ctypes.c_uint64 * 2)(1, 2)
    b = (ctypes.c_uint8 * 100)()
    data = (ctypes.c_void_p * 2)(ctypes.addressof(b), ctypes.addressof(b))
    lens = (ctypes.c_uint32 * 2)(100, 100)
    out = (ctypes.c_uint8 * (100 * 64))()
    desc = (L.PacketDesc * 64)()
    n_out = (ctypes.c_uint32 * 2)()
    cap = lib.qf_adaptive_max_send_packets(f.handle)
    # out_cap below the sum of max_send_packets: nothing consumed
    s = lib.qf_adaptive_on_send_batch(conns, 2, ids, data, lens, out, 100, None, 0, desc, 2 * cap - 1, n_out, None)
    assert s == L.QF_ETOOSMALL
    lens[1] = 101   # longer than max_len
    assert lib.qf_adaptive_on_send_batch(conns, 2, ids, data, lens, out, 100, None, 0, desc, 64, n_out,
                                         None) == L.QF_EINVAL
    lens[1] = 100   # repairs need out_stride >= max_len
    assert lib.qf_adaptive_on_send_batch(conns, 2, ids, data, lens, out, 99, None, 0, desc, 64, n_out,
                                         None) == L.QF_EINVAL
    assert lib.qf_adaptive_on_send_batch(conns, 0, None, None, None, None, 0, None, 0, None, 0, None, None) == 0
    # the failed calls left the window empty: a twin that saw nothing agrees
    twin = qf.AdaptiveFec(_cfg(qf, qf.FecMode.Light, max_len=100), now=0.0)
    k = f.state()["k"]
    for i in range(k):
        q1, _ = qf.on_send_batch([f], [qf.Packet(i, bytearray([i] * 10), 10, True)])
        q2 = []
        twin.on_send(qf.Packet(i, bytearray([i] * 10), 10, True), q2)
        assert len(q1[0]) == len(q2) and all(_same(a, b) for a, b in zip(q1[0], q2))
    assert len(q1[0]) > 1


def test_send_batch_second_context(qf, oracle, gpu_ctx):
    """A connection on another context takes the per-connection path inside
    the batch; every connection equals its twin."""
    ctx2 = qf.Context(0)
    cfg = _cfg(qf, qf.FecMode.Normal, normal_window=20, max_len=600)
    conns = [qf.AdaptiveFec(cfg, now=0.0), qf.AdaptiveFec(cfg, now=0.0, ctx=ctx2), qf.AdaptiveFec(cfg, now=0.0)]
    twins = [qf.AdaptiveFec(cfg, now=0.0) for _ in conns]
    rng = np.random.default_rng(3)
    for i in range(25):
        pays = [rng.integers(0, 256, 600, dtype=np.uint8).tobytes() for _ in conns]
        q, st = qf.on_send_batch(conns, [qf.Packet(i, bytearray(b), 600, True) for b in pays])
        for c in range(3):
            want = []
            twins[c].on_send(qf.Packet(i, bytearray(pays[c]), 600, True), want)
            assert st[c] == L.QF_OK and len(q[c]) == len(want) and all(_same(a, b) for a, b in zip(q[c], want))


def test_send_batch_after_per_packet_sends(qf, oracle, gpu_ctx):
    """A connection driven alternately by per-packet on_send (whose window-
    completing packet waits for the fused send kernel) and by send batches
    (which upload any waiting packet before their ring scatter) emits exactly
    what its per-packet twin emits, and every repair matches the oracle."""
    cfg = _cfg(qf, qf.FecMode.Normal, normal_window=16, max_len=600)
    a, twin = _pair(qf, cfg)
    other, other_twin = _pair(qf, cfg)
    rng = np.random.default_rng(3)
    hist = []
    k = a.state()["k"]
    r = a.state()["n"] - k
    for t in range(60):
        ln = int(rng.integers(1, 600))
        b = rng.integers(0, 256, ln, dtype=np.uint8).tobytes()
        b2 = rng.integers(0, 256, ln, dtype=np.uint8).tobytes()
        hist.append(b)
        want, want2 = [], []
        twin.on_send(qf.Packet(t, bytearray(b), ln, True), want)
        other_twin.on_send(qf.Packet(t, bytearray(b2), ln, True), want2)
        if t % 4 in (1, 2):     # per-packet
            got, got2 = [], []
            a.on_send(qf.Packet(t, bytearray(b), ln, True), got)
            other.on_send(qf.Packet(t, bytearray(b2), ln, True), got2)
        else:                   # one batch of both connections
            outs, st = qf.on_send_batch([a, other], [qf.Packet(t, bytearray(b), ln, True),
                                                     qf.Packet(t, bytearray(b2), ln, True)])
            assert st == [L.QF_OK, L.QF_OK]
            got, got2 = outs[0], outs[1]
        assert len(got) == len(want) and all(_same(p, q) for p, q in zip(got, want)), t
        assert len(got2) == len(want2) and all(_same(p, q) for p, q in zip(got2, want2)), t
        reps = [p for p in got if not p.is_systematic]
        if reps:
            _check_oracle(oracle, k, r, hist, reps)


@pytest.mark.parametrize("encode_small", [1, 0])
def test_send_batch_bursts(qf, oracle, gpu_ctx, encode_small):
    """One connection's burst in one call (the connection repeated B times,
    B = 1 .. 200, from an empty window and across k): its windows overlap and
    go to the device in one launch from a staging area holding the ring's
    newest k - 1 rows and the burst.  Everything equals the per-packet twin,
    every repair the oracle's encode of its window, and the ring left behind
    serves the next call (per-packet and batched).  encode_small = 0: the
    double ring of the bit-sliced per-packet path."""
    ctx = qf.Context(0)
    ctx.set_option("encode_small", encode_small)
    M = qf.FecMode
    cfgs = {"normal": _cfg(qf, M.Normal, normal_window=20, max_len=700), "light": _cfg(qf, M.Light, max_len=700)}
    conns = {n: qf.AdaptiveFec(c, now=0.0, ctx=ctx) for n, c in cfgs.items()}
    twins = {n: qf.AdaptiveFec(c, now=0.0, ctx=ctx) for n, c in cfgs.items()}
    single, single_twin = qf.AdaptiveFec(cfgs["normal"], now=0.0, ctx=ctx), qf.AdaptiveFec(cfgs["normal"], now=0.0, ctx=ctx)
    rng = np.random.default_rng(29)
    hist = {n: [] for n in conns}
    hist["single"] = []
    nid = {"normal": 0, "light": 10 ** 6, "single": 2 * 10 ** 6}
    n_checked = 0
    for B in (1, 5, 3, 16, 17, 40, 1, 200, 2, 64):
        order = ["normal"] * B + ["light"] * (B // 2 + 1) + ["single"]
        order = [order[i] for i in rng.permutation(len(order))]
        fecs, pkts = [], []
        for n in order:
            ln = int(rng.integers(0, 701)) if rng.random() < 0.3 else 700
            b = rng.integers(0, 256, ln, dtype=np.uint8).tobytes()
            fecs.append(single if n == "single" else conns[n])
            pkts.append((n, qf.Packet(nid[n], bytearray(b), ln, True)))
            nid[n] += 1
        if B == 2:   # a per-packet send between bursts reads the ring the burst left
            for n in ("normal", "light"):
                b = rng.integers(0, 256, 700, dtype=np.uint8).tobytes()
                got, want = [], []
                conns[n].on_send(qf.Packet(nid[n], bytearray(b), 700, True), got)
                twins[n].on_send(qf.Packet(nid[n], bytearray(b), 700, True), want)
                nid[n] += 1
                hist[n].append(b)
                assert len(got) == len(want) and all(_same(a, c) for a, c in zip(got, want))
        queues, st = qf.on_send_batch(fecs, [p for _, p in pkts])
        assert st == [L.QF_OK] * len(fecs)
        for m, (n, p) in enumerate(pkts):
            want = []
            tw = single_twin if n == "single" else twins[n]
            tw.on_send(qf.Packet(p.id, bytearray(p.payload()), p.len, True), want)
            assert len(queues[m]) == len(want), (B, n, m)
            assert all(_same(a, c) for a, c in zip(queues[m], want)), (B, n, m)
            hist[n].append(p.payload())
            f = single if n == "single" else conns[n]
            k, nn = f.state()["k"], f.state()["n"]
            if len(queues[m]) > 1 and (m % 5 == 0 or B < 20):
                _check_oracle(oracle, k, nn - k, hist[n], queues[m][1:])
                n_checked += 1
    assert n_checked > 40
