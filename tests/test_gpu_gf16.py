"""GF(2^16) Extreme mode on the MI355X (k_matvec16 / k_decode16_prepare / the
large-erasure path) against the oracle (oracle/qf_oracle16.c: Encoder16 and
Decoder16 of decoder.rs:10-88, 536-656 with the intended reduction) and the
reference's contract tests/fec.rs:52-82.  Bit-exact."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _r16(x):
    return (x + 15) // 16 * 16


def run_encode16(qf, src, r, coeff=None):
    """src: (G, k, L) -> (G, r, L); padded strides, guard bytes checked."""
    import torch

    G, k, L = src.shape
    rs, rrs = _r16(L) + 16, _r16(L) + 32
    gs, rgs = k * rs + 16, r * rrs + 48
    host = np.zeros(G * gs, np.uint8)
    for g in range(G):
        for i in range(k):
            host[g * gs + i * rs: g * gs + i * rs + L] = src[g, i]
    t_src = torch.from_numpy(host).to("cuda")
    t_rep = torch.full((G * rgs + 64,), 0xA5, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    qf.encode16_batch(t_src, t_rep, k, r, L, src_row_stride=rs, src_gen_stride=gs, rep_row_stride=rrs,
                      rep_gen_stride=rgs, G=G, coeff=coeff)
    qf.default_context().sync()
    out = t_rep.cpu().numpy()
    rep = np.zeros((G, r, L), np.uint8)
    guard = np.ones(out.shape, bool)
    for g in range(G):
        for j in range(r):
            o = g * rgs + j * rrs
            rep[g, j] = out[o: o + L]
            guard[o: o + L] = False
    assert (out[guard] == 0xA5).all(), "encode16 wrote outside [0, L) of a repair row"
    return rep


@pytest.mark.parametrize("k,r,L,G", [(8, 4, 8, 1), (1, 1, 2, 3), (16, 9, 100, 4), (64, 16, 1200, 6),
                                     (5, 17, 34, 2), (300, 8, 258, 2)])
def test_encode16_matches_oracle(qf, oracle, gpu_ctx, k, r, L, G):
    rng = np.random.default_rng(k * 1000 + r)
    src = rng.integers(0, 256, (G, k, L), dtype=np.uint8)
    src[0, 0, :4] = 0  # zero symbols (no log)
    rep = run_encode16(qf, src, r)
    for g in range(G):
        assert np.array_equal(rep[g], oracle.encode16(src[g], r)), g


def test_encode16_explicit_coefficients(qf, oracle, gpu_ctx):
    rng = np.random.default_rng(11)
    k, r, L = 12, 5, 66
    src = rng.integers(0, 256, (2, k, L), dtype=np.uint8)
    C = rng.integers(0, 65536, (r, k), dtype=np.uint16)
    C[0, :3] = 0
    C[1, 0] = 1
    rep = run_encode16(qf, src, r, coeff=C.tolist())
    for g in range(2):
        assert np.array_equal(rep[g], oracle.encode16(src[g], r, C))


def test_encode16_odd_length_rejected(qf, gpu_ctx):
    import torch

    t = torch.zeros(64, dtype=torch.uint8, device="cuda")
    with pytest.raises(qf.QfError):
        qf.encode16_batch(t, t, 2, 1, 3, src_row_stride=16, src_gen_stride=32, rep_row_stride=16,
                          rep_gen_stride=16, G=1)


def make_gens(oracle, rng, k, r, L, G, *, coeff_mode="cauchy", erase=None, dup=False, short=False):
    src = rng.integers(0, 256, (G, k, L), dtype=np.uint8)
    gens = []
    for g in range(G):
        C = oracle.cauchy16(k, r) if coeff_mode == "cauchy" else rng.integers(1, 65536, (r, k), dtype=np.uint16)
        rep = oracle.encode16(src[g], r, C)
        e = int(rng.integers(0, min(k, r) + 1)) if erase is None else erase
        er = set(rng.choice(k, e, replace=False).tolist())
        arr = [i for i in range(k) if i not in er]
        rng.shuffle(arr)
        reps = [k + j for j in rng.permutation(r)[:e].tolist()]
        arr = arr + reps + [k + j for j in range(r) if k + j not in reps]
        first = arr[:k]  # the first k rows are the system, in a random order
        rng.shuffle(first)
        arr = first + arr[k:]
        if dup and k > 1:
            arr.insert(1, arr[0])
        if short:
            arr = arr[: k - 1]
        rows = np.stack([src[g, a] if a < k else rep[a - k] for a in arr])
        rc = np.stack([np.zeros(k, np.uint16) if a < k else C[a - k] for a in arr])
        gens.append((arr, rows, rc))
    return src, gens


def run_decode16(qf, k, r, L, G, gens, with_coeffs):
    import torch

    max_rows = max(len(a) for a, _, _ in gens)
    rs = _r16(L) + 16
    rgs = max_rows * rs
    emax = min(k, r)
    rrs = _r16(L) + 16
    rec_gs = emax * rrs + 32
    rows = np.zeros(G * rgs, np.uint8)
    ridx = np.zeros((G, max_rows), np.uint16)
    nrows = np.zeros(G, np.uint32)
    rcoef = np.zeros((G, max_rows, k), np.uint16)
    for g, (arr, rw, rc) in enumerate(gens):
        nrows[g] = len(arr)
        ridx[g, : len(arr)] = arr
        for s in range(len(arr)):
            rows[g * rgs + s * rs: g * rgs + s * rs + L] = rw[s]
        rcoef[g, : len(arr)] = rc
    t_rows = torch.from_numpy(rows).to("cuda")
    t_idx = torch.from_numpy(ridx.view(np.int16)).to("cuda")
    t_n = torch.from_numpy(nrows.view(np.int32)).to("cuda")
    t_coef = torch.from_numpy(rcoef.view(np.int16).reshape(-1)).to("cuda") if with_coeffs else None
    t_rec = torch.full((G * rec_gs + 64,), 0x5A, dtype=torch.uint8, device="cuda")
    t_ri = torch.zeros(G * emax, dtype=torch.int16, device="cuda")
    t_nrec = torch.zeros(G, dtype=torch.int32, device="cuda")
    t_st = torch.full((G,), 77, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    qf.decode16_batch(t_rows, t_idx, t_rec, t_ri, t_nrec, t_st, k, r, L, max_rows=max_rows, row_stride=rs,
                      rows_gen_stride=rgs, rec_row_stride=rrs, rec_gen_stride=rec_gs, G=G, n_rows=t_n,
                      row_coeffs=t_coef)
    qf.default_context().sync()
    return (t_rec.cpu().numpy(), t_ri.cpu().numpy().view(np.uint16).reshape(G, emax), t_nrec.cpu().numpy(),
            t_st.cpu().numpy(), rrs, rec_gs)


def check_decode(oracle, src, gens, k, L, res):
    rec, ri, nrec, st, rrs, rec_gs = res
    for g, (arr, rows, rc) in enumerate(gens):
        ost, out, mask = oracle.decode16(k, arr, rows, rc if any(a >= k for a in arr) else None)
        assert st[g] == ost, (g, st[g], ost)
        if ost != 0:
            assert nrec[g] == 0
            continue
        erased = [i for i in range(k) if not mask[i]]
        assert nrec[g] == len(erased)
        assert ri[g, : len(erased)].tolist() == erased
        for b, i in enumerate(erased):
            o = g * rec_gs + b * rrs
            got = rec[o: o + L]
            assert np.array_equal(got, out[i]), (g, i)
            assert np.array_equal(got, src[g, i]), (g, i)


@pytest.mark.parametrize("lds_gj", ["0", "1"])
@pytest.mark.parametrize("k,r,L,G,with_coeffs", [(8, 4, 8, 5, False), (16, 16, 100, 8, False),
                                                 (64, 16, 1200, 12, False), (64, 64, 258, 4, False),
                                                 (10, 6, 34, 6, True), (40, 20, 66, 4, True)])
def test_decode16_small_path(qf, oracle, gpu_ctx, k, r, L, G, with_coeffs, lds_gj, monkeypatch):
    """Both decode paths for e <= 64: syndromes + closed-form / workspace
    inverse (default) and the all-generations Gauss-Jordan in LDS."""
    qf.set_default_options(gf16_lds_gj=int(lds_gj))
    rng = np.random.default_rng(k * 7 + r)
    src, gens = make_gens(oracle, rng, k, r, L, G, coeff_mode="cauchy" if not with_coeffs else "random")
    check_decode(oracle, src, gens, k, L, run_decode16(qf, k, r, L, G, gens, with_coeffs))


@pytest.mark.parametrize("lds_gj", ["0", "1"])
def test_decode16_statuses(qf, oracle, gpu_ctx, lds_gj, monkeypatch):
    qf.set_default_options(gf16_lds_gj=int(lds_gj))
    rng = np.random.default_rng(5)
    k, r, L = 12, 6, 40
    _, g1 = make_gens(oracle, rng, k, r, L, 1, erase=3, short=True)   # ENOTREADY
    _, g2 = make_gens(oracle, rng, k, r, L, 1, erase=3, dup=True)     # duplicated row: singular
    src, g3 = make_gens(oracle, rng, k, r, L, 1, erase=6)
    gens = g1 + g2 + g3
    srcs = np.concatenate([np.zeros((2, k, L), np.uint8), src])
    res = run_decode16(qf, k, r, L, 3, gens, False)
    assert res[3].tolist()[:2] == [-3, -4]
    check_decode(oracle, srcs, gens, k, L, res)


@pytest.mark.parametrize("dyn", ["1", "0"])
@pytest.mark.parametrize("lds_gj", ["0", "1"])
def test_decode16_mixed_erasures_device_shape(qf, oracle, gpu_ctx, lds_gj, dyn, monkeypatch):
    """Generations with very different e in one batch (0, a few, e_max, a
    short and a singular one): the split matvecs are shaped on the device from
    the largest e_g (k_shape16), the rows of every generation still match."""
    qf.set_default_options(gf16_lds_gj=int(lds_gj))
    qf.set_default_options(gf16_dyn=int(dyn))   # 0: the host's e_max shape
    rng = np.random.default_rng(17)
    k, r, L = 128, 64, 200
    parts = [make_gens(oracle, rng, k, r, L, 1, erase=e) for e in (0, 3, 64, 17)]
    parts.append(make_gens(oracle, rng, k, r, L, 1, erase=5, short=True))
    parts.append(make_gens(oracle, rng, k, r, L, 1, erase=9, dup=True))
    src = np.concatenate([p[0] for p in parts])
    gens = [p[1][0] for p in parts]
    res = run_decode16(qf, k, r, L, len(gens), gens, False)
    assert res[3][4] == -3 and (res[3][:4] == 0).all()   # short: ENOTREADY; the dup one per the oracle
    check_decode(oracle, src, gens, k, L, res)


@pytest.mark.parametrize("k,r,L,erase,with_coeffs", [(128, 96, 200, 80, False), (256, 128, 130, 128, False),
                                                     (160, 80, 66, 70, True)])
def test_decode16_large_path(qf, oracle, gpu_ctx, k, r, L, erase, with_coeffs):
    rng = np.random.default_rng(k + erase)
    src, gens = make_gens(oracle, rng, k, r, L, 2, coeff_mode="random" if with_coeffs else "cauchy", erase=erase)
    check_decode(oracle, src, gens, k, L, run_decode16(qf, k, r, L, 2, gens, with_coeffs))


def test_decode16_extreme_window_roundtrip(qf, oracle, gpu_ctx):
    """An Extreme-mode window (adaptive.rs:131: 1024..4096): k = 1024 sources,
    half erased, recovered from Cauchy repairs; checked against the sources
    (size-independent property: decode(encode(x)) == x)."""
    rng = np.random.default_rng(21)
    k, r, L, e = 1024, 1024, 256, 512
    src = rng.integers(0, 256, (1, k, L), dtype=np.uint8)
    rep = run_encode16(qf, src, r)[0]
    er = sorted(rng.choice(k, e, replace=False).tolist())
    arr = [i for i in range(k) if i not in set(er)] + [k + j for j in rng.permutation(r)[:e].tolist()]
    rng.shuffle(arr)
    rows = np.stack([src[0, a] if a < k else rep[a - k] for a in arr])
    rc = np.zeros((len(arr), k), np.uint16)
    rec, ri, nrec, st, rrs, rec_gs = run_decode16(qf, k, r, L, 1, [(arr, rows, rc)], False)
    assert st[0] == 0 and nrec[0] == e
    assert ri[0, :e].tolist() == er
    for b, i in enumerate(er):
        assert np.array_equal(rec[b * rrs: b * rrs + L], src[0, i])


def test_reference_contract_gf16_encode_decode(qf, gpu_ctx):
    """tests/fec.rs:52-82 through Encoder16 / Decoder16: k = 8, n = 12, packet
    0 dropped, every source's first byte comes back (the whole generation)."""
    k, n, L = 8, 12, 8
    enc = qf.Encoder16(k, n)
    pk = [qf.Packet(i, bytearray([i % 255] * L), L, True) for i in range(k)]
    for p in pk:
        enc.add_source_packet(p)
    repairs = [enc.generate_repair_packet(j) for j in range(n - k)]
    assert all(p is not None and p.coeff_len == 2 * k for p in repairs)
    dec = qf.Decoder16(k)
    for p in pk[1:] + repairs:
        dec.add_packet(p)
    assert dec.is_decoded
    out = dec.get_decoded_packets()
    assert len(out) == k
    assert [p.data[0] for p in out] == [i % 255 for i in range(k)]
    assert dec.get_decoded_packets() == []  # take()n


def test_encoder16_window_and_odd_length(qf, oracle, gpu_ctx):
    """Encoder16 (decoder.rs:25-75): None until the window is full, the window
    slides, repair j = Cauchy row y = k + j over the window in order, id =
    last.id + 1 + j, and an odd length leaves the last repair byte 0."""
    k, L = 6, 11
    rng = np.random.default_rng(2)
    src = rng.integers(0, 256, (k + 4, L), dtype=np.uint8)
    enc = qf.Encoder16(k, k + 3)
    for i in range(k + 4):
        if i < k:
            assert enc.generate_repair_packet(0) is None
        enc.add_source_packet(qf.Packet(100 + i, bytearray(src[i].tobytes()), L, True))
    win = src[4:]
    want = oracle.encode16(np.ascontiguousarray(win[:, : L - 1]), 3)
    for j in range(3):
        p = enc.generate_repair_packet(j)
        assert p.id == 100 + k + 3 + 1 + j and p.len == L
        assert p.payload()[: L - 1] == want[j].tobytes() and p.payload()[L - 1] == 0


def test_decoder16_reference_shapes(qf, gpu_ctx):
    """tests/fec.rs:128-228 (gf16_large_window / gf16_window_1024) drop a third
    / half of the sources but send only 8 repairs, so fewer than k rows arrive
    and the generation cannot decode; those tests' success assertions are
    unsatisfiable (as tests/high_loss.rs).  The decoder reports not
    decoded; with enough repairs the same shape decodes."""
    for k, keep in ((512, lambda i: i % 3 != 0), (1024, lambda i: i % 2 == 0)):
        L = 16
        enc = qf.Encoder16(k, k + 8)
        pk = [qf.Packet(i, bytearray([i % 255] * L), L, True) for i in range(k)]
        for p in pk:
            enc.add_source_packet(p)
        dec = qf.Decoder16(k)
        for p in [p for i, p in enumerate(pk) if keep(i)] + [enc.generate_repair_packet(j) for j in range(8)]:
            dec.add_packet(p)
        assert not dec.is_decoded and dec.get_decoded_packets() == []
    k = 512
    enc = qf.Encoder16(k, 2 * k)
    pk = [qf.Packet(i, bytearray([i % 255] * 16), 16, True) for i in range(k)]
    for p in pk:
        enc.add_source_packet(p)
    dec = qf.Decoder16(k)
    kept = [p for i, p in enumerate(pk) if i % 3 != 0]
    for p in kept + enc.generate_repairs(0, k - len(kept)):
        dec.add_packet(p)
    assert dec.is_decoded
    assert [p.data[0] for p in dec.get_decoded_packets()] == [i % 255 for i in range(k)]


@pytest.mark.parametrize("k,r,L,G", [(64, 16, 1200, 40), (64, 16, 1194, 7), (16, 4, 34, 5), (32, 8, 100, 3),
                                     (16, 4, 2, 9), (64, 16, 16, 300)])
def test_encode16_bitsliced(qf, oracle, gpu_ctx, k, r, L, G):
    """The generated bit-sliced kernel (qf_gf16_bs.hip) runs for the plain
    Cauchy batch of its (k, r), bit-exact against the oracle, including the
    partial last unit (L % 16 != 0) and lanes past the row; the general
    k_matvec16 path (gf16_bitsliced = 0) gives the same bytes."""
    from quicfuscate_amd import gf16_codegen as g16

    rng = np.random.default_rng(k * 7 + L)
    src = rng.integers(0, 256, (G, k, L), dtype=np.uint8)
    src[0, 0, :4] = 0
    gpu_ctx.profile(True)
    rep = run_encode16(qf, src, r)
    names = set(gpu_ctx.kernel_times())
    gpu_ctx.profile(False)
    assert g16.kernel_name(k, r) in names, names
    for g in range(G):
        assert np.array_equal(rep[g], oracle.encode16(src[g], r)), g
    qf.set_default_options(gf16_bitsliced=0)
    rep2 = run_encode16(qf, src, r)
    assert np.array_equal(rep, rep2)


@pytest.mark.parametrize("L", [1200, 1194])
def test_decode16_bitsliced_syndromes(qf, oracle, gpu_ctx, L):
    """Cauchy decode of a (k, r) with a generated bit-sliced kernel: the
    syndromes come from qf_gf16bs_syn_* (sources gathered through the slot
    map, the accepted repair row XORed in), the general matvec only for the
    generation with a repair index past k + r; statuses, recovered bytes and
    indices equal the oracle's and the general path's (gf16_bitsliced = 0).
    At L % 16 != 0 the bit-sliced kernel (whole 16-B units, up to 15 bytes
    past the last row) is not used: the other path, same bytes."""
    from quicfuscate_amd import gf16_codegen as g16

    k, r = 64, 16
    rng = np.random.default_rng(1616)
    src, gens = make_gens(oracle, rng, k, r, L, 8)
    _, full = make_gens(oracle, rng, k, r, L, 1, erase=16)
    _, none = make_gens(oracle, rng, k, r, L, 1, erase=0)
    _, short = make_gens(oracle, rng, k, r, L, 1, erase=5, short=True)
    _, dup = make_gens(oracle, rng, k, r, L, 1, erase=3, dup=True)
    src = np.concatenate([src, src[:4]])
    gens += [full[0], none[0], short[0], dup[0]]
    # generation 0: one accepted repair row is Cauchy row k + 20 (no row of the kernel)
    arr, rows, rc = gens[0]
    far = oracle.encode16(src[0], 21)[20]
    pos = next(s for s, a in enumerate(arr[:k]) if a < k)
    gens[0] = ([k + 20] + [a for s, a in enumerate(arr) if s != pos],
               np.concatenate([far[None], np.delete(rows, pos, 0)]), None)
    G = len(gens)
    src_used = np.stack([src[g] for g in range(8)] + [np.zeros((k, L), np.uint8)] * 4)
    gpu_ctx.profile(True)
    res = run_decode16(qf, k, r, L, G, [(a, rw, np.zeros((len(a), k), np.uint16)) for a, rw, _ in gens], False)
    names = set(gpu_ctx.kernel_times())
    gpu_ctx.profile(False)
    if L % 16 == 0:
        assert g16.kernel_name(k, r, "syn") in names and "k_syndromes16_fallback" in names, names
    else:
        assert g16.kernel_name(k, r, "syn") not in names, names
    rec, ri, nrec, st, rrs, rec_gs = res
    for g, (a, rw, _) in enumerate(gens):
        ost, out, mask = oracle.decode16(k, a, rw, None)
        assert st[g] == ost, (g, st[g], ost)
        if ost:
            assert nrec[g] == 0
            continue
        erased = [i for i in range(k) if not mask[i]]
        assert nrec[g] == len(erased) and ri[g, : len(erased)].tolist() == erased, g
        for b, i in enumerate(erased):
            o = g * rec_gs + b * rrs
            assert np.array_equal(rec[o: o + L], out[i]), (g, i)
    qf.set_default_options(gf16_bitsliced=0)
    res2 = run_decode16(qf, k, r, L, G, [(a, rw, np.zeros((len(a), k), np.uint16)) for a, rw, _ in gens], False)
    for x, y in zip(res[:4], res2[:4]):
        assert np.array_equal(x, y)


@pytest.mark.parametrize("k,r,L,G", [(16, 5, 100, 3), (32, 32, 2, 4), (128, 96, 200, 2), (256, 1, 34, 5),
                                     (1024, 1024, 64, 1), (1024, 8, 1200, 2), (4096, 100, 32, 1),
                                     (4096, 16, 4, 1), (2048, 2048, 100, 3), (64, 33, 1200, 9),
                                     (256, 200, 9000, 2)])
@pytest.mark.parametrize("bs", [2, 3, 0])
def test_encode16_fft(qf, oracle, gpu_ctx, k, r, L, G, bs):
    """Power-of-two windows without a bit-sliced kernel run the additive-FFT
    kernel (qf_gf16_fft.hip; bs 2 / 3: the bit-plane kernel for k <= 2,048,
    one / two layers per LDS pass, bs 0: the log / Zech one): bit-exact against the oracle's Encoder16 and
    against the general k_matvec16 path (gf16_fft = 0); guard bytes outside
    [0, L) of every repair row untouched (run_encode16)."""
    rng = np.random.default_rng(k * 13 + r + L)
    src = rng.integers(0, 256, (G, k, L), dtype=np.uint8)
    src[0, 0, :4] = 0
    src[-1, -1, -2:] = 0
    qf.set_default_options(gf16_fft=2, gf16_fft_bs=bs)   # the FFT wherever it applies
    gpu_ctx.profile(True)
    rep = run_encode16(qf, src, r)
    names = set(gpu_ctx.kernel_times())
    gpu_ctx.profile(False)
    assert "k_fft16_encode" in names, names
    for g in range(G):
        assert np.array_equal(rep[g], oracle.encode16(src[g], r)), g
    if k <= 1024:
        qf.set_default_options(gf16_fft=0)
        assert np.array_equal(rep, run_encode16(qf, src, r))


def test_encode16_fft_many_generations(qf, oracle, gpu_ctx):
    """More generations than one launch's grid.y (65,535): sampled generations
    against the oracle."""
    import torch

    k, r, L, G = 16, 3, 16, 70000
    rng = np.random.default_rng(70000)
    src = rng.integers(0, 256, (G, k, L), dtype=np.uint8)
    t_src = torch.from_numpy(src.reshape(-1)).to("cuda")
    t_rep = torch.zeros(G * r * 16, dtype=torch.uint8, device="cuda")
    qf.set_default_options(gf16_fft=2)
    qf.encode16_batch(t_src, t_rep, k, r, L, src_row_stride=L, src_gen_stride=k * L, rep_row_stride=16,
                      rep_gen_stride=r * 16, G=G)
    qf.default_context().sync()
    rep = t_rep.cpu().numpy().reshape(G, r, 16)[:, :, :L]
    for g in [0, 1, 65534, 65535, 65536, 69999] + rng.integers(0, G, 20).tolist():
        assert np.array_equal(rep[g], oracle.encode16(src[g], r)), g


@pytest.mark.parametrize("bs", [2, 3, 0])
def test_encoder16_fft_window_slides(qf, oracle, gpu_ctx, bs):
    """Encoder16 over a power-of-two window (decoder.rs:25-75): after the
    window slides (ring rotation) and for a repair range starting past 0, the
    FFT kernel's repairs equal the oracle's Cauchy rows over the window."""
    k, L = 64, 40
    rng = np.random.default_rng(64)
    src = rng.integers(0, 256, (k + 5, L), dtype=np.uint8)
    enc = qf.Encoder16(k, k + 12)
    for i in range(k + 5):
        enc.add_source_packet(qf.Packet(i, bytearray(src[i].tobytes()), L, True))
    want = oracle.encode16(np.ascontiguousarray(src[5:]), 12)
    C = oracle.cauchy16(k, 12)
    qf.set_default_options(gf16_fft=2, gf16_fft_bs=bs)
    gpu_ctx.profile(True)
    got = [enc.generate_repair_packet(j) for j in (0, 7)] + enc.generate_repairs(3, 9)
    names = set(gpu_ctx.kernel_times())
    gpu_ctx.profile(False)
    assert "k_fft16_encode" in names, names
    assert got[0].payload() == want[0].tobytes() and got[1].payload() == want[7].tobytes()
    for n, p in enumerate(got[2:]):
        assert p.payload() == want[3 + n].tobytes(), n
        assert p.coeff_len == 2 * k
        assert bytes(p.coefficients[: 2 * k]) == np.asarray(C[3 + n], dtype=">u2").tobytes(), n


@pytest.mark.parametrize("k,r,L", [(128, 40, 100), (256, 256, 34), (32, 16, 2), (1024, 16, 66)])
@pytest.mark.parametrize("bs", [2, 3, 0])
def test_decode16_fft_syndromes(qf, oracle, gpu_ctx, k, r, L, bs):
    """Cauchy decode of a power-of-two k without a bit-sliced kernel: the
    syndromes come from the additive FFT (k_fft16_syndromes, sources gathered
    through the slot map, erased ones as zero rows, the accepted repair row
    XORed in), the general matvec only for the generation with a repair index
    past k + r; the solve x_E = C[J,E]^-1 s is the FFT too (k_fft16_solve),
    the matvec only for a repair index >= 2k (k = r = 256); statuses, recovered bytes and indices equal the oracle's and
    the general path's (gf16_fft = 0).  Mixed erasure counts, a full-erasure,
    an erasure-free, a short and a duplicate-row generation."""
    rng = np.random.default_rng(k + r + L)
    src, gens = make_gens(oracle, rng, k, r, L, 6)
    e_full = min(k, r)
    _, full = make_gens(oracle, rng, k, r, L, 1, erase=e_full)
    _, none = make_gens(oracle, rng, k, r, L, 1, erase=0)
    _, short = make_gens(oracle, rng, k, r, L, 1, erase=min(5, e_full), short=True)
    _, dup = make_gens(oracle, rng, k, r, L, 1, erase=min(3, e_full), dup=True)
    src = np.concatenate([src, src[:4]])
    gens += [full[0], none[0], short[0], dup[0]]
    # generation 0: one accepted repair row is Cauchy row k + r + 3 (past the FFT's coset rows)
    arr, rows, rc = gens[0]
    extra = r + 3
    if k + extra < 65536 and any(a < k for a in arr[:k]):
        far = oracle.encode16(src[0], extra + 1)[extra]
        pos = next(s for s, a in enumerate(arr[:k]) if a < k)
        gens[0] = ([k + extra] + [a for s, a in enumerate(arr) if s != pos],
                   np.concatenate([far[None], np.delete(rows, pos, 0)]), None)
    G = len(gens)
    qf.set_default_options(gf16_fft=2, gf16_fft_bs=bs)
    gpu_ctx.profile(True)
    res = run_decode16(qf, k, r, L, G, [(a, rw, np.zeros((len(a), k), np.uint16)) for a, rw, _ in gens], False)
    names = set(gpu_ctx.kernel_times())
    gpu_ctx.profile(False)
    assert "k_fft16_syndromes" in names and "k_syndromes16_fallback" in names, names
    assert "k_fft16_solve" in names, names
    rec, ri, nrec, st, rrs, rec_gs = res
    for g, (a, rw, _) in enumerate(gens):
        ost, out, mask = oracle.decode16(k, a, rw, None)
        assert st[g] == ost, (g, st[g], ost)
        if ost:
            assert nrec[g] == 0
            continue
        erased = [i for i in range(k) if not mask[i]]
        assert nrec[g] == len(erased) and ri[g, : len(erased)].tolist() == erased, g
        for b, i in enumerate(erased):
            o = g * rec_gs + b * rrs
            assert np.array_equal(rec[o: o + L], out[i]), (g, i)
    qf.set_default_options(gf16_fft=0)
    res2 = run_decode16(qf, k, r, L, G, [(a, rw, np.zeros((len(a), k), np.uint16)) for a, rw, _ in gens], False)
    for x, y in zip(res[:4], res2[:4]):
        assert np.array_equal(x, y)


@pytest.mark.parametrize("k,r,L,e", [(2048, 64, 40, 64), (1024, 1024, 34, 700), (2048, 2048, 6, 1500)])
def test_decode16_fft_large_windows(qf, oracle, gpu_ctx, k, r, L, e):
    """Extreme-size windows (the oracle's k^3 elimination is too slow here):
    every erased source comes back equal to the source row, and the bit-plane
    FFT kernels (k <= 2,048: 1,024-thread variant at k = 2,048) give the same
    bytes, statuses and indices as the log / Zech kernels."""
    rng = np.random.default_rng(k + r + L + e)
    src, gens = make_gens(oracle, rng, k, r, L, 2, erase=e)
    G = len(gens)
    out = {}
    for bs in (2, 3, 0):
        qf.set_default_options(gf16_fft=2, gf16_fft_bs=bs)
        gpu_ctx.profile(True)
        out[bs] = run_decode16(qf, k, r, L, G, [(a, rw, np.zeros((len(a), k), np.uint16)) for a, rw, _ in gens],
                               False)
        names = set(gpu_ctx.kernel_times())
        gpu_ctx.profile(False)
        assert "k_fft16_syndromes" in names and "k_fft16_solve" in names, names
    rec, ri, nrec, st, rrs, rec_gs = out[2]
    for g, (a, rw, _) in enumerate(gens):
        assert st[g] == 0
        erased = sorted(set(range(k)) - set(x for x in a[:k] if x < k))
        assert nrec[g] == len(erased) == e and ri[g, :e].tolist() == erased, g
        for b, i in enumerate(erased):
            o = g * rec_gs + b * rrs
            assert np.array_equal(rec[o: o + L], src[g, i]), (g, i)
    for bs in (3, 0):
        for x, y in zip(out[2][:4], out[bs][:4]):
            assert np.array_equal(x, y), bs
