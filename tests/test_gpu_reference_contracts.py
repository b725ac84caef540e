"""The reference's own FEC tests, restated through the Python mirror of its
API (quicfuscate_amd.fec), running on the MI355X library.

tests/fec.rs and src/fec/mod.rs build packets with make_packet(id, val):
8 bytes of `val` in a pool block (tests/fec.rs:5-18) and assert that
out[i].data[0] == i after encode/erase/decode."""
import pytest

pytestmark = pytest.mark.gpu


def make_packet(qf, pid, val, pool):
    buf = pool.alloc()
    buf[:8] = bytes([val & 0xFF]) * 8
    return qf.Packet(pid, buf, 8, True)


def _roundtrip(qf, k, n, keep_src, keep_rep, val=lambda i: i):
    qf.init_gf_tables()
    pool = qf.MemoryPool(64, 64)
    enc = qf.Encoder(k, n, max_len=64)
    packets = []
    for i in range(k):
        p = make_packet(qf, i, val(i), pool)
        enc.add_source_packet(p.clone())
        packets.append(p)
    repairs = [enc.generate_repair_packet(i, pool) for i in range(n - k)]
    assert all(r is not None for r in repairs)
    dec = qf.Decoder(k, pool)
    for i, p in enumerate(packets):
        if keep_src(i):
            dec.add_packet(p.clone())
    for j, r in enumerate(repairs):
        if keep_rep(j):
            dec.add_packet(r)
    return dec, packets, repairs


def test_gf8_encode_decode(qf, gpu_ctx):
    # tests/fec.rs:20-50
    dec, _, _ = _roundtrip(qf, 4, 6, lambda i: i != 1, lambda j: True)
    assert dec.is_decoded
    out = dec.get_decoded_packets()
    assert len(out) == 4
    for i in range(4):
        assert out[i].data[0] == i
        assert bytes(out[i].data[:8]) == bytes([i]) * 8


def test_gaussian_path_decodes(qf, gpu_ctx):
    # src/fec/mod.rs:107-139 (drop packet 2)
    dec, _, _ = _roundtrip(qf, 4, 6, lambda i: i != 2, lambda j: True)
    assert dec.is_decoded
    out = dec.get_decoded_packets()
    assert [p.data[0] for p in out] == [0, 1, 2, 3]


def test_repair_known_answer(qf, gpu_ctx):
    # SURVEY 8(c) KAT: repairs of the k=4 make_packet window are [128]*8, [160]*8
    _, _, repairs = _roundtrip(qf, 4, 6, lambda i: True, lambda j: False)
    assert bytes(repairs[0].data[:8]) == bytes([128]) * 8
    assert bytes(repairs[1].data[:8]) == bytes([160]) * 8
    assert repairs[0].coefficients == bytes([71, 167, 122, 186])
    assert repairs[0].id == 3 + 1 + 0 and repairs[1].id == 3 + 1 + 1   # decoder.rs:267


def test_recovery_low_loss(qf, gpu_ctx):
    # src/fec/mod.rs:295-322
    dec, _, _ = _roundtrip(qf, 10, 12, lambda i: i != 3, lambda j: True)
    assert dec.is_decoded


def test_recovery_high_loss(qf, gpu_ctx):
    # src/fec/mod.rs:324-353
    dec, _, _ = _roundtrip(qf, 16, 32, lambda i: i % 2 == 0, lambda j: j % 3 != 0, val=lambda i: i % 255)
    assert dec.is_decoded
    out = dec.get_decoded_packets()
    assert [p.data[0] for p in out] == list(range(16))
    assert dec.get_decoded_packets() == []  # drained (take())


def test_window_not_full_returns_none(qf, gpu_ctx):
    # decoder.rs:177-179
    pool = qf.MemoryPool(8, 64)
    enc = qf.Encoder(4, 6, max_len=64)
    enc.add_source_packet(make_packet(qf, 0, 0, pool))
    assert enc.generate_repair_packet(0, pool) is None


def test_sliding_window_slides(qf, oracle, gpu_ctx):
    # decoder.rs:164-169: the oldest packet leaves once k are held
    import numpy as np

    pool = qf.MemoryPool(8, 64)
    enc = qf.Encoder(4, 5, max_len=64)
    for i in range(7):
        enc.add_source_packet(make_packet(qf, i, 10 + i, pool))
    rep = enc.generate_repair_packet(0, pool)
    window = np.stack([np.full(8, 10 + i, np.uint8) for i in range(3, 7)])
    assert bytes(rep.data[:8]) == oracle.encode(window, 1)[0].tobytes()
    assert rep.id == 6 + 1


def test_repair_without_coefficients_is_an_error(qf, gpu_ctx):
    # decoder.rs:699 Err("Repair packet missing coefficients.")
    dec = qf.Decoder(4, qf.MemoryPool(8, 64))
    with pytest.raises(qf.QfError):
        dec.add_packet(qf.Packet(9, bytearray(8), 8, False))


def test_duplicate_systematic_ignored(qf, gpu_ctx):
    # decoder.rs:687-691
    pool = qf.MemoryPool(16, 64)
    dec = qf.Decoder(4, pool)
    p = make_packet(qf, 1, 1, pool)
    assert not dec.add_packet(p.clone())
    assert not dec.add_packet(p.clone())
    for i in (0, 2, 3):
        dec.add_packet(make_packet(qf, i, i, pool))
    assert dec.is_decoded


@pytest.mark.parametrize("k,n", [(1024, 1032), (512, 516), (260, 264)])
def test_large_windows_error_where_reference_panics(qf, gpu_ctx, k, n):
    # tests/fec.rs:94-126, 162-194; mod.rs:141-175: k + r > 256 panics in
    # gf_inv(0) -> QF_ERANGE (or EINVAL for k > 256 windows).
    with pytest.raises(qf.QfError):
        enc = qf.Encoder(k, n, max_len=16)
        pool = qf.MemoryPool(k, 16)
        for i in range(k):
            enc.add_source_packet(qf.Packet(i, bytearray(8), 8, True))
        enc.generate_repair_packet(0, pool)


def test_empty_and_degenerate_batches(qf, gpu_ctx):
    """Empty inputs are no-ops that touch no memory (null buffers allowed);
    malformed shapes are QF_EINVAL, never a fault (SURVEY 8(b) errors)."""
    from quicfuscate_amd import _lib as L

    lib, h = L._lib(), gpu_ctx.handle
    enc = lambda k, r, Lb, G, flags=0: lib.qf_encode_batch(  # noqa: E731
        h, L.EncodeShape(k, r, Lb, flags, Lb, k * Lb, Lb, r * Lb), G, None, None, None)
    assert enc(64, 16, 1200, 0) == 0          # G = 0
    assert enc(64, 0, 1200, 4) == 0           # r = 0: nothing to emit
    assert enc(64, 16, 0, 4) == 0             # L = 0: empty payloads
    assert enc(0, 16, 1200, 4) == L.QF_EINVAL
    assert enc(257, 1, 1200, 4) == L.QF_EINVAL
    assert enc(64, 16, 1200, 4, flags=0x80) == L.QF_EINVAL
    assert enc(64, 16, 1200, 4) == L.QF_EINVAL  # G > 0 with null buffers
    dec = lambda k, r, Lb, mr, G: lib.qf_decode_batch(  # noqa: E731
        h, L.DecodeShape(k, r, Lb, mr, Lb, mr * Lb, Lb, r * Lb), G, None, None, None, None, None, None,
        None, None)
    assert dec(64, 16, 1200, 80, 0) == 0      # G = 0
    assert dec(64, 16, 0, 80, 1) == L.QF_EINVAL
    assert dec(64, 16, 1200, 0, 1) == L.QF_EINVAL
    assert dec(0, 16, 1200, 80, 1) == L.QF_EINVAL
    assert dec(64, 16, 1200, 80, 1) == L.QF_EINVAL  # G > 0 with null buffers
    gpu_ctx.sync()


def test_decoded_packet_ids_follow_reference_rule(qf, gpu_ctx):
    """decoder.rs:688 / 771: a received systematic packet keeps its own id; a
    reconstructed one gets id = i.  Stream ids that are not 0..k-1 (here
    1000..) must survive the decode unchanged."""
    k, n = 8, 12
    pool = qf.MemoryPool(32, 64)
    enc = qf.Encoder(k, n, max_len=64)
    pk = []
    for i in range(k):
        p = make_packet(qf, 1000 + i, 40 + i, pool)   # 1000 % 8 == 0: column i
        enc.add_source_packet(p.clone())
        pk.append(p)
    reps = [enc.generate_repair_packet(j, pool) for j in range(n - k)]
    lost = {2, 5}
    dec = qf.Decoder(k, pool)
    for i, p in enumerate(pk):
        if i not in lost:
            dec.add_packet(p.clone())
    for rp in reps[: len(lost)]:
        dec.add_packet(rp)
    assert dec.is_decoded
    out = dec.get_decoded_packets()
    assert [p.id for p in out] == [i if i in lost else 1000 + i for i in range(k)]
    assert [p.data[0] for p in out] == [40 + i for i in range(k)]


@pytest.mark.parametrize("small", ["1", "0"])
@pytest.mark.parametrize("k", [16, 64, 128])
def test_ring_encoder_every_rotation(qf, oracle, gpu_ctx, monkeypatch, small, k):
    """The encoder object's window lives in a ring read rotated by the
    small-batch kernel (QF_ENCODE_SMALL=1) or doubled for the bit-sliced
    kernels (=0).  After 3k packets every rotation has been passed; the
    repairs of each window must equal the oracle's encode of the last k
    packets (decoder.rs:164-275)."""
    import numpy as np

    qf.set_default_options(encode_small=int(small))
    Lb, r = 1200, 4
    enc = qf.Encoder(k, k + r, max_len=Lb)
    rng = np.random.default_rng(k)
    data = rng.integers(0, 256, (3 * k, Lb), dtype=np.uint8)
    pool = qf.MemoryPool(4, Lb)
    checked = 0
    for t in range(3 * k):
        enc.add_source_packet(qf.Packet(t, bytearray(data[t].tobytes()), Lb, True))
        if t + 1 < k or (t % 7 != 3 and t != 3 * k - 1):
            continue
        want = oracle.encode(data[t + 1 - k: t + 1], r)
        for j in range(r):
            rp = enc.generate_repair_packet(j, pool)
            assert bytes(rp.data[:Lb]) == want[j].tobytes(), (t, j)
            assert rp.id == t + 1 + j
        checked += 1
    assert checked >= 6


@pytest.mark.parametrize("fused", ["1", "0"])
@pytest.mark.parametrize("k,max_len", [(16, 1500), (64, 1200), (5, 9000)])
def test_fused_send_window(qf, oracle, gpu_ctx, monkeypatch, fused, k, max_len):
    """The packet that completes a window waits on the host and travels in
    the arguments of the one fused send kernel (QF_SEND_FUSED, default on;
    not above 3,584-byte slots).  Repairs of every window equal the oracle's
    encode of the last k packets, with window[0].len != the new packet's len
    (decoder.rs:172-275), a first repair other than 0, a generate without
    output bytes (the packet is uploaded instead), and adds that skip the
    generate entirely."""
    import numpy as np

    qf.set_default_options(send_fused=int(fused))
    r = 3
    enc = qf.Encoder(k, k + r, max_len=max_len)
    rng = np.random.default_rng(k + max_len)
    pool = qf.MemoryPool(4, max_len)
    lens = [int(x) for x in rng.integers(1, max_len + 1, 3 * k)]
    data = [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in lens]
    for t in range(3 * k):
        enc.add_source_packet(qf.Packet(t, bytearray(data[t]), lens[t], True))
        if t + 1 < k or t % 3 == 1:
            continue                    # the next add uploads the waiting packet
        L = lens[t + 1 - k]
        window = np.zeros((k, L), np.uint8)
        for i in range(k):
            b = np.frombuffer(data[t + 1 - k + i], np.uint8)[:L]
            window[i, : len(b)] = b
        want = oracle.encode(window, r)
        if t % 6 == 5:   # no output bytes: the waiting packet is uploaded instead
            from quicfuscate_amd import _lib as LL
            assert LL._lib().qf_encoder_generate_repairs(enc.handle, 0, 1, None, 0, None, None, None) == 0
        j0 = 2 if t % 3 == 2 else 0     # a first repair other than 0 may consume the packet
        for j in list(range(j0, r)) + list(range(0, j0)):
            rp = enc.generate_repair_packet(j, pool)
            assert rp.len == L and bytes(rp.data[:L]) == want[j].tobytes(), (t, j)
            assert rp.id == t + 1 + j


def test_last_error_on_the_device(qf):
    """On a GPU host: an out-of-range device ordinal names hipErrorInvalidDevice;
    a decode that succeeds afterwards does not clear it (errno semantics)."""
    import ctypes
    from quicfuscate_amd import _lib as L

    lib = L._lib()
    h = ctypes.c_void_p()
    assert lib.qf_ctx_create(1 << 20, None, ctypes.byref(h)) == L.QF_EDEVICE
    why = lib.qf_last_error().decode()
    assert why.startswith("qf_api.hip:") and "hipErrorInvalidDevice" in why, why
    with pytest.raises(L.QfError) as ei:
        qf.check(lib.qf_ctx_create(1 << 20, None, ctypes.byref(h)), "ctx")
    assert "hipErrorInvalidDevice" in str(ei.value)
