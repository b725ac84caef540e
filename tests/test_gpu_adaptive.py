"""Adaptive FEC driver with its GF(2^8) codec on the device: per-packet
sliding-window repairs (adaptive.rs:519-562) equal the oracle's encode of
the window, and a receiver recovers the generation (adaptive.rs:566-599)."""
import numpy as np
import pytest

from quicfuscate_amd import _lib as L

pytestmark = pytest.mark.gpu


def _sender_receiver(qf, mode, max_len=1500):
    cfg = qf.FecConfig(initial_mode=mode, max_len=max_len)
    return qf.AdaptiveFec(cfg, now=0.0), qf.AdaptiveFec(cfg, now=0.0)


@pytest.mark.parametrize("mode,L_", [("Light", 8), ("Normal", 1200)])
def test_sliding_window_repairs_and_recovery(qf, oracle, gpu_ctx, mode, L_):
    M = qf.FecMode
    snd, rcv = _sender_receiver(qf, M[mode])
    k, n = snd.state()["k"], snd.state()["n"]
    r = n - k
    rng = np.random.default_rng(k)
    src = rng.integers(0, 256, (k + 3, L_), dtype=np.uint8)
    if mode == "Light":
        src[:] = np.arange(k + 3, dtype=np.uint8)[:, None]  # tests/fec.rs make_packet payloads [i]*8
    C = oracle.cauchy(k, r)
    out_all = []
    for i in range(k + 3):
        out = []
        s = snd.on_send(qf.Packet(i, bytearray(src[i].tobytes()), L_, True), out)
        assert s == L.QF_OK
        assert out[0].is_systematic and out[0].id == i and out[0].payload() == src[i].tobytes()
        reps = out[1:]
        if i < k - 1:
            assert reps == []          # window not full: generate_repair_packet -> None
            continue
        assert len(reps) == r
        want = oracle.encode(src[i - k + 1: i + 1], r)   # window = last k packets, oldest first
        for j, p in enumerate(reps):
            assert not p.is_systematic and p.id == i + 1 + j          # decoder.rs:265-273
            assert p.coeff_len == k and bytes(p.coefficients) == bytes(C[j])
            assert p.payload() == want[j].tobytes(), (i, j)
        out_all.append((i, out))
    # receiver: generation of packets 0..k-1 with 3 sources lost, repairs of that window
    i0, first = out_all[0]
    lost = {1, k // 2, k - 2}
    got = []
    for p in [qf.Packet(i, bytearray(src[i].tobytes()), L_, True) for i in range(k) if i not in lost] + first[1:]:
        got += rcv.on_receive(p)
    if r < len(lost):
        assert got == []
        return
    assert [p.id for p in got] == list(range(k))
    for p in got:
        assert p.payload() == src[p.id].tobytes()


def test_strong_mode_has_no_gf256_code(qf, gpu_ctx):
    # Strong's default window 512 -> (512, 768): the reference panics in
    # gf_inv(0); here the systematic packet goes out + QF_ERANGE
    snd = qf.AdaptiveFec(qf.FecConfig(initial_mode=qf.FecMode.Strong), now=0.0)
    out = []
    assert snd.on_send(qf.Packet(0, bytearray(b"abcdefgh"), 8, True), out) == L.QF_ERANGE
    assert len(out) == 1 and out[0].payload() == b"abcdefgh"


def test_cross_fade_with_codecs(qf, gpu_ctx):
    # Normal -> (PID as written) Medium with window 109 at t = 1 s; both
    # configurations take every packet during the fade
    snd = qf.AdaptiveFec(qf.FecConfig(initial_mode=qf.FecMode.Normal, pid=qf.PidConfig(1.0, 0.0, 0.0),
                                      lambda_=0.01, burst_window=50), now=0.0)
    snd.report_loss(0, 20, now=1.0)
    st = snd.state()
    assert st["mode"] == qf.FecMode.Medium and st["k"] == 109 and st["n"] == 142 and st["transitioning"]
    for i in range(40):
        out = []
        assert snd.on_send(qf.Packet(i, bytearray([i % 256] * 16), 16, True), out) == L.QF_OK
        assert len(out) == 1      # neither window (64 / 109 packets) is full yet
    assert not snd.is_transitioning()


@pytest.mark.parametrize("window,L_,lost", [(24, 40, (0, 5, 23)), (1024, 64, tuple(range(0, 1024, 9)))])
def test_extreme_mode_gf16_codec(qf, oracle, gpu_ctx, window, L_, lost):
    """Extreme mode runs the GF(2^16) codec (decoder.rs:96-102, 125-131):
    sliding-window repairs equal the GF(2^16) oracle's encode of the window
    with 2k-byte big-endian coefficient blocks, and a receiver recovers the
    generation through Decoder16 (closed-form path: aligned-window Cauchy rows)."""
    M = qf.FecMode
    wins = qf.default_windows()
    wins[M.Extreme] = window
    cfg = qf.FecConfig(initial_mode=M.Extreme, max_len=1500, window_sizes=wins)
    snd, rcv = qf.AdaptiveFec(cfg, now=0.0), qf.AdaptiveFec(cfg, now=0.0)
    k, n = snd.state()["k"], snd.state()["n"]
    assert (k, n) == (window, 2 * window)
    r = n - k
    rng = np.random.default_rng(window)
    src = rng.integers(0, 256, (k, L_), dtype=np.uint8)
    reps = None
    for i in range(k):
        out = []
        assert snd.on_send(qf.Packet(i, bytearray(src[i].tobytes()), L_, True), out) == L.QF_OK
        assert out[0].is_systematic and out[0].payload() == src[i].tobytes()
        if i < k - 1:
            assert len(out) == 1
        else:
            reps = out[1:]
    assert len(reps) == r
    C = oracle.cauchy16(k, r)
    check = sorted(set([0, 1, r - 1] + rng.integers(0, r, 5).tolist()))
    want = oracle.encode16(src, r, C[check])   # every window size, k = 1,024 included
    for q, j in enumerate(check):
        p = reps[j]
        assert not p.is_systematic and p.id == k + j and p.coeff_len == 2 * k
        assert bytes(p.coefficients) == b"".join(int(c).to_bytes(2, "big") for c in C[j])
        assert p.payload() == want[q].tobytes(), j
    got = []
    for p in [qf.Packet(i, bytearray(src[i].tobytes()), L_, True) for i in range(k) if i not in set(lost)] + reps:
        got += rcv.on_receive(p)
    assert [p.id for p in got] == list(range(k))
    for p in got:
        assert p.payload() == src[p.id].tobytes(), p.id
