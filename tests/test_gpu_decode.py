"""Decode parity on the MI355X: k_decode_prepare + k_combine_slots vs the
CPU oracle (decoder.rs:658-791 with the F4 fix).  Recovered rows must be the
original source bytes and equal the oracle's solution; statuses must match
(ENOTREADY, ERANK)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _r16(x):
    return (x + 15) // 16 * 16


def make_batch(oracle, rng, k, r, L, G, max_rows, *, dup_prob=0.0, shuffle=True, erase=None,
               coeff_mode="cauchy", trim_prob=0.0):
    """Per generation: source rows, repairs, an arrival list (row index per slot)."""
    src = rng.integers(0, 256, (G, k, L), dtype=np.uint8)
    gens = []
    for g in range(G):
        if coeff_mode == "cauchy":
            C = oracle.cauchy(k, r)
        else:
            C = rng.integers(0, 256, (r, k), dtype=np.uint8)
        rep = oracle.encode(src[g], r, C)
        e = rng.integers(0, min(k, r) + 1) if erase is None else erase
        erased = set(rng.choice(k, size=e, replace=False).tolist())
        arr = [i for i in range(k) if i not in erased] + [k + j for j in range(r)]
        if shuffle:
            rng.shuffle(arr)
        if dup_prob:
            extra = [a for a in arr if rng.random() < dup_prob]
            for a in extra:
                arr.insert(int(rng.integers(0, len(arr) + 1)), a)
        arr = arr[:max_rows]
        if trim_prob and rng.random() < trim_prob:  # fewer rows than needed -> ENOTREADY
            arr = arr[: int(rng.integers(0, k))]
        rows = np.stack([src[g, a] if a < k else rep[a - k] for a in arr]) if arr else np.zeros((0, L), np.uint8)
        rc = np.stack([np.zeros(k, np.uint8) if a < k else C[a - k] for a in arr]) if arr else None
        gens.append((arr, rows, rc))
    return src, gens


def run_decode(qf, k, r, L, G, max_rows, gens, with_coeffs):
    import torch

    rs = _r16(L) + 16
    rgs = max_rows * rs
    emax = min(k, r)
    rrs = _r16(L) + 16
    rec_gs = emax * rrs + 32
    rows = np.zeros(G * rgs, np.uint8)
    ridx = np.zeros((G, max_rows), np.uint16)
    nrows = np.zeros(G, np.uint32)
    rcoef = np.zeros((G, max_rows, k), np.uint8)
    for g, (arr, rw, rc) in enumerate(gens):
        nrows[g] = len(arr)
        ridx[g, : len(arr)] = arr
        for s in range(len(arr)):
            rows[g * rgs + s * rs: g * rgs + s * rs + L] = rw[s]
            if rc is not None:
                rcoef[g, s] = rc[s]
    dev = "cuda"
    t_rows = torch.from_numpy(rows).to(dev)
    t_idx = torch.from_numpy(ridx.view(np.int16)).to(dev)
    t_n = torch.from_numpy(nrows.view(np.int32)).to(dev)
    t_coef = torch.from_numpy(rcoef.reshape(-1)).to(dev) if with_coeffs else None
    t_rec = torch.full((G * rec_gs + 64,), 0x5A, dtype=torch.uint8, device=dev)
    t_recidx = torch.zeros(G * max(emax, 1), dtype=torch.int16, device=dev)
    t_nrec = torch.zeros(G, dtype=torch.int32, device=dev)
    t_status = torch.full((G,), 77, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    qf.decode_batch(t_rows, t_idx, t_rec, t_recidx, t_nrec, t_status, k, r, L, max_rows=max_rows,
                    row_stride=rs, rows_gen_stride=rgs, rec_row_stride=rrs, rec_gen_stride=rec_gs,
                    G=G, n_rows=t_n, row_coeffs=t_coef)
    qf.default_context().sync()
    return (t_rec.cpu().numpy(), t_recidx.cpu().numpy().view(np.uint16).reshape(G, -1),
            t_nrec.cpu().numpy(), t_status.cpu().numpy(), rrs, rec_gs)


def check(oracle, k, L, src, gens, out, with_coeffs):
    rec, recidx, nrec, status, rrs, rec_gs = out
    for g, (arr, rw, rc) in enumerate(gens):
        st, sol, mask = oracle.decode(k, arr, rw if len(arr) else np.zeros((0, L), np.uint8),
                                      rc if with_coeffs else None)
        assert status[g] == st, (g, status[g], st)
        if st != 0:
            assert nrec[g] == 0
            continue
        erased = [i for i in range(k) if not mask[i]]
        assert nrec[g] == len(erased)
        assert list(recidx[g, : nrec[g]]) == erased
        for m, i in enumerate(erased):
            got = rec[g * rec_gs + m * rrs: g * rec_gs + m * rrs + L]
            assert (got == sol[i]).all(), (g, i)
            assert (got == src[g, i]).all(), (g, i)
            assert (rec[g * rec_gs + m * rrs + L: g * rec_gs + (m + 1) * rrs] == 0x5A).all()


PATHS = ["default", "default_1wave", "default_nofft", "default_waveprep", "syn", "general", "syn_bs", "general_bs"]


def _path(_unused, path):
    """Pin the decode path on the default context (fec.set_default_options;
    conftest restores the options after each test)."""
    from quicfuscate_amd import fec

    # "default" at these batch sizes (at most one item per CU) runs the
    # row-split kernels (qf_cauchy_decs_*, and qf_cauchy_bss_* for the r > 16
    # syndrome passes: four waves per item); "default_1wave" pins the
    # one-wave-per-item kernels (qf_cauchy_decc_*, qf_cauchy_bs_*)
    # (and the payload pass k_combine_slots_split against k_combine_slots)
    # "default_nofft": the one-wave kernels with one coefficient block per
    # repair instead of the additive-FFT row loop (QF_OPT_FFT_KERNELS = 0)
    # "default_waveprep": the one-wave kernels with the acceptance pass one
    # generation per wave (k_decode_prepare_lu) instead of per lane
    one = path in ("default_1wave", "default_nofft", "default_waveprep")
    fft = 0 if path == "default_nofft" else 1
    lanes = 0 if path == "default_waveprep" else 1
    if one:
        path = "default"
    opts = dict(decode_ksplit=0 if one else 1, encode_ksplit=0 if one else 1, combine_split=0 if one else 1,
                fft_kernels=fft, prepare_lanes=lanes)
    # "*_bs": the payload pass takes the bit-sliced qf_combine_bs at every row
    # length (by default only rows of >= 64 lane-chunks of 32 B do); "general"
    # keeps k_combine_slots at every length (combine_bs 0)
    opts.update(combine_bs=1, combine_bs_min_q=64)
    if path.endswith("_bs"):
        opts["combine_bs_min_q"] = 1
        path = path[:-3]
    elif path == "general":
        opts["combine_bs"] = 0
    # "default": fused decode (syndromes + LU solve in one kernel) where a
    # bit-sliced kernel exists for (k, r) (Cauchy code, L % 16 == 0);
    # "syn": syndrome kernel + payload pass (two kernels);
    # "general": Gauss-Jordan + payload pass
    opts["bitsliced"] = 0 if path == "general" else 1
    opts["decode_path"] = 1 if path == "syn" else 0
    fec.set_default_options(**opts)


@pytest.mark.parametrize("path", PATHS)
@pytest.mark.parametrize("k,r,L,G", [(64, 16, 1200, 40), (16, 16, 100, 30), (4, 2, 8, 20),
                                     (10, 2, 8, 20), (33, 7, 37, 25), (1, 3, 16, 10),
                                     (16, 16, 96, 30), (32, 16, 64, 25), (64, 10, 1216, 20),
                                     (16, 1, 64, 40), (64, 16, 80, 50),
                                     # C5 shapes with generated kernels; 9000: partial last unit
                                     (32, 5, 1200, 30), (48, 8, 1200, 30), (96, 15, 1200, 20),
                                     (96, 15, 9000, 4), (48, 8, 1000, 12),
                                     # r > 16: syndromes through the encode kernels, passes of 16 outputs
                                     (128, 20, 1200, 8), (128, 39, 1000, 6), (160, 48, 700, 4),
                                     (196, 59, 9000, 2)])
def test_decode_matches_oracle_random_erasures(qf, oracle, gpu_ctx, k, r, L, G, path, monkeypatch):
    _path(monkeypatch, path)
    rng = np.random.default_rng(k + r + L)
    max_rows = k + r
    src, gens = make_batch(oracle, rng, k, r, L, G, max_rows)
    out = run_decode(qf, k, r, L, G, max_rows, gens, False)
    check(oracle, k, L, src, gens, out, False)


@pytest.mark.parametrize("path", PATHS)
def test_decode_cauchy_duplicates_and_short_generations(qf, oracle, gpu_ctx, path, monkeypatch):
    # duplicated sources (counted once) and repairs (singular -> ERANK), and
    # generations with fewer than k rows (ENOTREADY), mixed in one batch
    _path(monkeypatch, path)
    rng = np.random.default_rng(99)
    k, r, L, G = 16, 16, 64, 120
    max_rows = 48
    src, gens = make_batch(oracle, rng, k, r, L, G, max_rows, dup_prob=0.08, trim_prob=0.15)
    out = run_decode(qf, k, r, L, G, max_rows, gens, False)
    check(oracle, k, L, src, gens, out, False)
    assert {0, -3, -4} <= set(out[3].tolist())


@pytest.mark.parametrize("path", PATHS)
def test_decode_bench_shape_fixed_13_erasures(qf, oracle, gpu_ctx, path, monkeypatch):
    _path(monkeypatch, path)
    # k=64, 13 erased sources, arrival = surviving sources then repairs
    rng = np.random.default_rng(2024)
    k, r, L, G = 64, 16, 1200, 24
    src, gens = make_batch(oracle, rng, k, r, L, G, k - 13 + r, shuffle=False, erase=13)
    out = run_decode(qf, k, r, L, G, k - 13 + r, gens, False)
    check(oracle, k, L, src, gens, out, False)


def test_decode_row_split_threshold(qf, oracle, gpu_ctx, monkeypatch):
    """The fused decode takes the row-split kernel (qf_cauchy_decs_*, four
    waves per item) up to one item per CU and the one-wave kernel
    (qf_cauchy_decc_*) beyond: both sides of the switch, bit-exact."""
    import torch

    _path(monkeypatch, "default")
    k, r, L = 64, 16, 1200
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    Q = ((L + 15) // 16 + 1) // 2          # lane-chunks per generation
    g_max = 64 * ncu // Q                  # largest G with ceil(G*Q/64) <= ncu
    ctx = qf.default_context()
    for G, want in ((g_max, "decs"), (g_max + 1, "decc")):
        rng = np.random.default_rng(G)
        src, gens = make_batch(oracle, rng, k, r, L, G, k - 13 + r, shuffle=False, erase=13)
        ctx.sync()
        ctx.profile(True)
        out = run_decode(qf, k, r, L, G, k - 13 + r, gens, False)
        names = set(ctx.kernel_times())
        ctx.profile(False)
        # (decc: the additive-FFT variant qf_cauchy_deccf8_* where generated)
        assert any(n.startswith(f"qf_cauchy_{want}") and n.endswith("_k64_r16") for n in names), (G, names)
        check(oracle, k, L, src, gens, out, False)


def test_decode_explicit_coefficients_and_duplicates(qf, oracle, gpu_ctx):
    # random coefficient matrices (some singular) + duplicate arrivals
    rng = np.random.default_rng(7)
    k, r, L, G = 12, 8, 64, 60
    max_rows = 40
    src, gens = make_batch(oracle, rng, k, r, L, G, max_rows, dup_prob=0.15, coeff_mode="random")
    out = run_decode(qf, k, r, L, G, max_rows, gens, True)
    check(oracle, k, L, src, gens, out, True)
    assert set(out[3].tolist()) >= {0}


def test_decode_repair_index_out_of_range(qf, oracle, gpu_ctx):
    # without row_coeffs a repair row's index must be < k + r (its Cauchy row)
    rng = np.random.default_rng(4)
    k, r, L = 16, 16, 64
    src = rng.integers(0, 256, (2, k, L), dtype=np.uint8)
    rep = oracle.encode(src[0], r)
    gens = [(list(range(1, k)) + [k + r], np.vstack([src[0, 1:], rep[:1]]), None),
            (list(range(k)), src[1], None)]
    for path in PATHS:
        qf.set_default_options(bitsliced=0 if path == "general" else 1)
        out = run_decode(qf, k, r, L, 2, k, gens, False)
        assert list(out[3]) == [-1, 0], path


def test_decode_not_enough_rows_and_singular(qf, oracle, gpu_ctx):
    rng = np.random.default_rng(3)
    k, r, L = 8, 4, 48
    src = rng.integers(0, 256, (3, k, L), dtype=np.uint8)
    C = oracle.cauchy(k, r)
    gens = []
    rep0 = oracle.encode(src[0], r)
    gens.append(([0, 1, 2, 8], np.vstack([src[0, :3], rep0[:1]]), None))             # ENOTREADY
    rep1 = oracle.encode(src[1], r)
    gens.append(([0, 1, 2, 3, 4, 5, 8, 8, 9], np.vstack([src[1, :6], rep1[0], rep1[0], rep1[1]]), None))  # ERANK
    rep2 = oracle.encode(src[2], r)
    gens.append(([8, 9, 10, 11, 0, 1, 2, 3, 4, 5], np.vstack([rep2, src[2, :6]]), None))  # OK, e = 4
    out = run_decode(qf, k, r, L, 3, 12, gens, False)
    check(oracle, k, L, src, gens, out, False)
    assert list(out[3]) == [-3, -4, 0]


def test_decode_many_erasures_multi_pass(qf, oracle, gpu_ctx):
    # e > 16 -> several 16-row payload passes
    rng = np.random.default_rng(11)
    k, r, L, G = 40, 40, 80, 12
    src, gens = make_batch(oracle, rng, k, r, L, G, k + r, erase=33)
    out = run_decode(qf, k, r, L, G, k + r, gens, False)
    check(oracle, k, L, src, gens, out, False)


def test_decode_no_erasures(qf, oracle, gpu_ctx):
    rng = np.random.default_rng(12)
    k, r, L, G = 16, 4, 32, 5
    src, gens = make_batch(oracle, rng, k, r, L, G, k + r, erase=0, shuffle=False)
    out = run_decode(qf, k, r, L, G, k + r, gens, False)
    check(oracle, k, L, src, gens, out, False)
    assert (out[2] == 0).all()


@pytest.mark.parametrize("chunk,overlap", [("7", "1"), ("7", "0"), ("16", "1")])
def test_decode_chunked_pipeline(qf, oracle, gpu_ctx, chunk, overlap, monkeypatch):
    # stages A/B over chunks of generations, B on an auxiliary stream
    # (double-buffered syndromes); twice in a row on the same context
    qf.set_default_options(decode_chunk=int(chunk), decode_overlap=int(overlap), decode_path=1, bitsliced=1)
    for seed in (1, 2):
        rng = np.random.default_rng(seed)
        k, r, L, G = 64, 16, 1200, 53
        src, gens = make_batch(oracle, rng, k, r, L, G, k + r, shuffle=True)
        out = run_decode(qf, k, r, L, G, k + r, gens, False)
        check(oracle, k, L, src, gens, out, False)


@pytest.mark.parametrize("path", PATHS)
def test_decode_payload_wait_orders_the_rows_copy(qf, oracle, gpu_ctx, path, monkeypatch):
    """qf_ctx_set_payload_wait: the rows land on another stream after a
    delay; the decode's payload pass must wait for that stream's event (the
    acceptance pass needs only the indices).  Without the gate it would read
    the 0xEE placeholder rows."""
    import torch

    _path(monkeypatch, path)
    k, r, L, G = 64, 16, 1200, 300
    max_rows = k + r
    rng = np.random.default_rng(11)
    src, gens = make_batch(oracle, rng, k, r, L, G, max_rows, erase=13)
    rs, emax = _r16(L), min(k, r)
    rgs, rec_gs = max_rows * rs, emax * rs
    rows = np.zeros(G * rgs, np.uint8)
    ridx = np.zeros((G, max_rows), np.uint16)
    nrows = np.zeros(G, np.uint32)
    for g, (arr, rw, _) in enumerate(gens):
        nrows[g] = len(arr)
        ridx[g, : len(arr)] = arr
        for s in range(len(arr)):
            rows[g * rgs + s * rs: g * rgs + s * rs + L] = rw[s]
    staged = torch.from_numpy(rows).cuda()
    t_rows = torch.full_like(staged, 0xEE)
    t_idx = torch.from_numpy(ridx.view(np.int16)).cuda()
    t_n = torch.from_numpy(nrows.view(np.int32)).cuda()
    t_rec = torch.zeros(G * rec_gs, dtype=torch.uint8, device="cuda")
    t_recidx = torch.zeros(G * emax, dtype=torch.int16, device="cuda")
    t_nrec = torch.zeros(G, dtype=torch.int32, device="cuda")
    t_status = torch.full((G,), 77, dtype=torch.int32, device="cuda")
    big_a = torch.ones(1 << 30, dtype=torch.uint8, device="cuda")
    big_b = torch.empty_like(big_a)
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    landed = torch.cuda.Event()
    with torch.cuda.stream(side):
        for _ in range(4):          # ~2 ms of HBM traffic ahead of the rows
            big_b.copy_(big_a)
        t_rows.copy_(staged)
        landed.record(side)
    ctx = qf.default_context()
    ctx.set_payload_wait(landed)
    qf.decode_batch(t_rows, t_idx, t_rec, t_recidx, t_nrec, t_status, k, r, L, max_rows=max_rows,
                    row_stride=rs, rows_gen_stride=rgs, rec_row_stride=rs, rec_gen_stride=rec_gs,
                    G=G, n_rows=t_n, ctx=ctx)
    ctx.sync()
    torch.cuda.synchronize()
    out = (t_rec.cpu().numpy(), t_recidx.cpu().numpy().view(np.uint16).reshape(G, -1),
           t_nrec.cpu().numpy(), t_status.cpu().numpy(), rs, rec_gs)
    assert (out[3] == 0).all()
    check(oracle, k, L, src, gens, out, False)
    # the gate is one call only: a plain decode afterwards runs unchanged
    ctx.set_payload_wait(None)
    del big_a, big_b


@pytest.mark.parametrize("k,r,L,G", [(64, 16, 1200, 3000), (20, 9, 200, 50), (128, 39, 9000, 24)])
def test_decode_payload_stream(qf, oracle, gpu_ctx, k, r, L, G):
    """qf_ctx_set_payload_stream: the acceptance pass stays on the context's
    stream, the payload pass (or, for paths that finish on the context's
    stream, a wait for them) is enqueued on the caller's stream, so work
    queued on that stream afterwards sees the recovered rows with no other
    synchronisation.  The setting holds for one decode call."""
    import torch

    max_rows = k + r
    rng = np.random.default_rng(k + r + L)
    src, gens = make_batch(oracle, rng, k, r, L, G, max_rows, erase=min(r, max(1, k // 5)))
    rs, emax = _r16(L), min(k, r)
    rgs, rec_gs = max_rows * rs, emax * rs
    rows = np.zeros(G * rgs, np.uint8)
    ridx = np.zeros((G, max_rows), np.uint16)
    nrows = np.zeros(G, np.uint32)
    for g, (arr, rw, _) in enumerate(gens):
        nrows[g] = len(arr)
        ridx[g, : len(arr)] = arr
        for s in range(len(arr)):
            rows[g * rgs + s * rs: g * rgs + s * rs + L] = rw[s]
    t_rows = torch.from_numpy(rows).cuda()
    t_idx = torch.from_numpy(ridx.view(np.int16)).cuda()
    t_n = torch.from_numpy(nrows.view(np.int32)).cuda()
    t_rec = torch.full((G * rec_gs,), 0x5A, dtype=torch.uint8, device="cuda")   # check(): bytes past L stay 0x5A
    t_recidx = torch.zeros(G * emax, dtype=torch.int16, device="cuda")
    t_nrec = torch.zeros(G, dtype=torch.int32, device="cuda")
    t_status = torch.full((G,), 77, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    ctx = qf.Context(0, torch.cuda.Stream().cuda_stream)     # the acceptance pass's own stream
    try:
        ctx.set_payload_stream(side)
        qf.decode_batch(t_rows, t_idx, t_rec, t_recidx, t_nrec, t_status, k, r, L, max_rows=max_rows,
                        row_stride=rs, rows_gen_stride=rgs, rec_row_stride=rs, rec_gen_stride=rec_gs,
                        G=G, n_rows=t_n, ctx=ctx)
        with torch.cuda.stream(side):      # ordered after the decode by the library alone
            snap = [t.clone() for t in (t_rec, t_recidx, t_nrec, t_status)]
        side.synchronize()
        out = (snap[0].cpu().numpy(), snap[1].cpu().numpy().view(np.uint16).reshape(G, -1),
               snap[2].cpu().numpy(), snap[3].cpu().numpy(), rs, rec_gs)
        assert (out[3] == 0).all()
        check(oracle, k, L, src, gens, out, False)
        ctx.sync()
    finally:
        ctx.close()


@pytest.mark.parametrize("path", PATHS)
@pytest.mark.parametrize("k,r,L,G,pin", [(64, 16, 1200, 2000, True), (16, 16, 100, 37, False),
                                         (96, 15, 9000, 120, True)])
def test_decode_batch_host_matches_oracle(qf, oracle, gpu_ctx, path, k, r, L, G, pin, monkeypatch):
    """qf_decode_batch_host: rows, indices and outputs in host memory,
    several pipelined chunks (k=64: ~96 KB per generation -> G=2000 spans 3
    chunks of 64 MiB); same results as the oracle."""
    import torch

    _path(monkeypatch, path)
    rng = np.random.default_rng(k * 7 + L)
    max_rows = k + r
    src, gens = make_batch(oracle, rng, k, r, L, G, max_rows, trim_prob=0.02)
    rs, emax = _r16(L), min(k, r)
    rgs, rec_gs = max_rows * rs, emax * rs
    rows = torch.zeros(G * rgs, dtype=torch.uint8, pin_memory=pin)
    rows_np = rows.numpy()
    ridx = np.zeros((G, max_rows), np.uint16)
    nrows = np.zeros(G, np.uint32)
    for g, (arr, rw, _) in enumerate(gens):
        nrows[g] = len(arr)
        ridx[g, : len(arr)] = arr
        for s in range(len(arr)):
            rows_np[g * rgs + s * rs: g * rgs + s * rs + L] = rw[s]
    t_idx = torch.from_numpy(ridx.view(np.int16).reshape(-1).copy())
    t_n = torch.from_numpy(nrows.view(np.int32).copy())
    t_rec = torch.full((G * rec_gs,), 0x5A, dtype=torch.uint8, pin_memory=pin)
    t_recidx = torch.zeros(G * emax, dtype=torch.int16, pin_memory=pin)
    t_nrec = torch.zeros(G, dtype=torch.int32, pin_memory=pin)
    t_status = torch.full((G,), 77, dtype=torch.int32, pin_memory=pin)
    qf.decode_batch_host(rows, t_idx, t_rec, t_recidx, t_nrec, t_status, k, r, L, max_rows=max_rows,
                         row_stride=rs, rows_gen_stride=rgs, rec_row_stride=rs, rec_gen_stride=rec_gs,
                         G=G, n_rows=t_n)
    out = (t_rec.numpy(), t_recidx.numpy().view(np.uint16).reshape(G, -1), t_nrec.numpy(), t_status.numpy(),
           rs, rec_gs)
    check(oracle, k, L, src, gens, out, False)


@pytest.mark.parametrize("k,r,L", [(64, 16, 48), (32, 5, 64), (96, 15, 32)])
def test_decode_prepare_per_lane_matches_per_wave(qf, oracle, gpu_ctx, k, r, L):
    """The acceptance pass one generation per lane (k_decode_prepare_lu_lanes,
    batches of >= 2,048 generations) against one per wave
    (k_decode_prepare_lu): duplicated sources and repairs, short generations,
    no erasures, every repair needed, repair indices out of range -- the
    recovered rows, indices, counts and statuses are identical, and every
    generation equals the oracle."""
    rng = np.random.default_rng(k * 7 + r)
    G = 2600
    max_rows = k + r + 4
    src, gens = make_batch(oracle, rng, k, r, L, G, max_rows, dup_prob=0.03, trim_prob=0.05)
    e_full = min(k, r)
    for g in range(0, G, 97):            # every repair needed
        _, full = make_batch(oracle, rng, k, r, L, 1, max_rows, erase=e_full)
        src[g] = _[0]
        gens[g] = full[0]
    for g in range(5, G, 101):           # no erasures
        _, none = make_batch(oracle, rng, k, r, L, 1, max_rows, erase=0)
        src[g] = _[0]
        gens[g] = none[0]
    bad = set(range(11, G, 211))         # a repair index past k + r: EINVAL
    for g in bad:
        arr, rows, rc = gens[g]
        if arr:
            arr = list(arr)
            arr[len(arr) // 2] = k + r + 3
            gens[g] = (arr, rows, rc)
    outs = {}
    for lanes in (1, 0):
        qf.set_default_options(prepare_lanes=lanes, decode_ksplit=0)
        outs[lanes] = run_decode(qf, k, r, L, G, max_rows, gens, False)
    for x, y in zip(outs[1][:4], outs[0][:4]):
        assert np.array_equal(x, y)
    status = outs[1][3]
    assert all(status[g] == -1 for g in bad if gens[g][0])
    assert {0, -1, -3, -4} <= set(status.tolist())
    good = [g for g in range(G) if g not in bad]
    rec, recidx, nrec, st, rrs, rec_gs = outs[1]
    for g in good:
        arr, rw, _ = gens[g]
        ost, sol, mask = oracle.decode(k, arr, rw if len(arr) else np.zeros((0, L), np.uint8), None)
        assert st[g] == ost, (g, st[g], ost)
        if ost:
            assert nrec[g] == 0
            continue
        erased = [i for i in range(k) if not mask[i]]
        assert nrec[g] == len(erased) and list(recidx[g, : nrec[g]]) == erased, g
        for m, i in enumerate(erased):
            assert (rec[g * rec_gs + m * rrs: g * rec_gs + m * rrs + L] == sol[i]).all(), (g, i)


def test_decode_payload_stream_back_to_back(qf, oracle, gpu_ctx):
    """two payload-stream decodes on one context, different rows,
    no join between them.  The first payload pass is held back on the caller's
    stream (HBM copies queued ahead of it); the second call's acceptance pass,
    on the context's stream, must not rewrite the context's LU records / slot
    map before that pass has read them."""
    import torch

    k, r, L, G = 64, 16, 1200, 3000
    max_rows = k + r
    rs, emax = _r16(L), min(k, r)
    rgs, rec_gs = max_rows * rs, emax * rs
    batches = []
    for seed in (21, 22):
        rng = np.random.default_rng(seed)
        src, gens = make_batch(oracle, rng, k, r, L, G, max_rows, erase=13)
        rows = np.zeros(G * rgs, np.uint8)
        ridx = np.zeros((G, max_rows), np.uint16)
        for g, (arr, rw, _) in enumerate(gens):
            ridx[g, : len(arr)] = arr
            for s in range(len(arr)):
                rows[g * rgs + s * rs: g * rgs + s * rs + L] = rw[s]
        t = dict(rows=torch.from_numpy(rows).cuda(), idx=torch.from_numpy(ridx.view(np.int16)).cuda(),
                 rec=torch.full((G * rec_gs,), 0x5A, dtype=torch.uint8, device="cuda"),
                 recidx=torch.zeros(G * emax, dtype=torch.int16, device="cuda"),
                 nrec=torch.zeros(G, dtype=torch.int32, device="cuda"),
                 status=torch.full((G,), 77, dtype=torch.int32, device="cuda"))
        batches.append((src, gens, t))
    big_a = torch.ones(1 << 30, dtype=torch.uint8, device="cuda")
    big_b = torch.empty_like(big_a)
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    ctx = qf.Context(0, torch.cuda.Stream().cuda_stream)
    try:
        with torch.cuda.stream(side):
            for _ in range(6):          # ~3 ms of HBM traffic ahead of the first payload pass
                big_b.copy_(big_a)
        for _, _, t in batches:
            ctx.set_payload_stream(side)
            qf.decode_batch(t["rows"], t["idx"], t["rec"], t["recidx"], t["nrec"], t["status"], k, r, L,
                            max_rows=max_rows, row_stride=rs, rows_gen_stride=rgs, rec_row_stride=rs,
                            rec_gen_stride=rec_gs, G=G, ctx=ctx)
        ctx.sync()          # the context's stream now also covers the payload passes
        for src, gens, t in batches:
            out = (t["rec"].cpu().numpy(), t["recidx"].cpu().numpy().view(np.uint16).reshape(G, -1),
                   t["nrec"].cpu().numpy(), t["status"].cpu().numpy(), rs, rec_gs)
            assert (out[3] == 0).all()
            check(oracle, k, L, src, gens, out, False)
    finally:
        ctx.close()
        del big_a, big_b


@pytest.mark.parametrize("path", ["default", "general"])
def test_decode_general_path_more_than_four_passes(qf, oracle, gpu_ctx, path, monkeypatch):
    """Cauchy k=128, r=96 (r > 64: no syndrome kernel) with 2 KiB
    rows takes the general path with the bit-sliced payload pass; e up to 96
    means up to 6 passes of 16 outputs, more than one pass-major launch holds,
    so the passes run one launch each instead of failing with QF_EDEVICE."""
    _path(monkeypatch, path)
    rng = np.random.default_rng(96)
    k, r, L, G = 128, 96, 2048, 4
    src, gens = make_batch(oracle, rng, k, r, L, G, k + r, erase=90)
    out = run_decode(qf, k, r, L, G, k + r, gens, False)
    check(oracle, k, L, src, gens, out, False)
    assert max(out[2]) > 64


@pytest.mark.parametrize("wide", [1, 0])
@pytest.mark.parametrize("path", ["default_1wave", "general_bs"])
@pytest.mark.parametrize("k,r,L,G,erase", [(128, 20, 9000, 5, None), (128, 20, 4100, 7, 20), (64, 24, 2048, 6, 24),
                                           (40, 20, 3000, 5, 17), (64, 24, 2100, 9, None)])
def test_decode_combine_wide(qf, oracle, gpu_ctx, k, r, L, G, erase, path, wide, monkeypatch):
    """A payload pass of 17-24 outputs (e_max = min(k, r)) as one 24-output
    pass reading two coefficient records per row (qf_combine_bs_r24,
    QF_OPT_COMBINE_WIDE = 1) or as two 16-output passes (0): bit-exact either
    way, on the C5 syndrome path and the general (Gauss-Jordan) path, with
    generations of e <= 16 (no pass-1 outputs) among them when e is random."""
    _path(monkeypatch, path)
    qf.set_default_options(combine_wide=wide)
    rng = np.random.default_rng(k * 7 + r + L + (erase or 0))
    kw = {"erase": erase, "shuffle": False} if erase is not None else {}
    max_rows = k + r
    src, gens = make_batch(oracle, rng, k, r, L, G, max_rows, **kw)
    out = run_decode(qf, k, r, L, G, max_rows, gens, False)
    check(oracle, k, L, src, gens, out, False)


@pytest.mark.parametrize("jump,xcd", [(1, 0), (0, 0), (1, 1), (0, 1)])
@pytest.mark.parametrize("path", ["default_1wave", "general_bs"])
@pytest.mark.parametrize("k,r,L,G,erase", [(196, 59, 9000, 5, None), (160, 48, 4100, 7, 40), (128, 39, 2100, 9, 30),
                                           (128, 20, 9000, 5, None), (64, 16, 3000, 6, 12)])
def test_decode_combine_jump_xcd(qf, oracle, gpu_ctx, k, r, L, G, erase, path, jump, xcd, monkeypatch):
    """The bit-sliced payload pass with its runtime-coefficient products as
    calls into per-coefficient code blocks (QF_OPT_COMBINE_JUMP = 1) or as
    M0-indexed XORs (0), pass-major or with the passes of a slot interleaved
    on one XCD (QF_OPT_COMBINE_XCD = 1): bit-exact in every combination, for
    one, two (wide), three and four passes, on the C5 syndrome path and the
    general (Gauss-Jordan) path."""
    _path(monkeypatch, path)
    qf.set_default_options(combine_jump=jump, combine_xcd=xcd)
    rng = np.random.default_rng(k * 11 + r + L + (erase or 0))
    kw = {"erase": erase, "shuffle": False} if erase is not None else {}
    max_rows = k + r
    src, gens = make_batch(oracle, rng, k, r, L, G, max_rows, **kw)
    out = run_decode(qf, k, r, L, G, max_rows, gens, False)
    check(oracle, k, L, src, gens, out, False)


@pytest.mark.parametrize("pm24", [1, 0])
@pytest.mark.parametrize("path", ["default_1wave", "general_bs"])
@pytest.mark.parametrize("k,r,L,G,erase", [(196, 59, 9000, 5, None), (196, 59, 4100, 6, 39), (160, 48, 4100, 7, 40),
                                           (128, 39, 2100, 9, 36), (100, 64, 3000, 5, None), (80, 40, 2500, 6, 33)])
def test_decode_combine_pm24(qf, oracle, gpu_ctx, k, r, L, G, erase, path, pm24, monkeypatch):
    """A payload pass of 33-64 outputs (e_max) as 24-output passes in one
    launch (qf_combine_bs_r24_pm_j3, QF_OPT_COMBINE_PM24 = 1; the last pass's
    pieces past the written records redirected) or as 16-output passes (0):
    bit-exact either way, random or fixed erasure counts, C5 and general
    paths, rows that end mid-unit."""
    _path(monkeypatch, path)
    qf.set_default_options(combine_pm24=pm24)
    rng = np.random.default_rng(k * 13 + r + L + (erase or 0))
    kw = {"erase": erase, "shuffle": False} if erase is not None else {}
    max_rows = k + r
    src, gens = make_batch(oracle, rng, k, r, L, G, max_rows, **kw)
    out = run_decode(qf, k, r, L, G, max_rows, gens, False)
    check(oracle, k, L, src, gens, out, False)


@pytest.mark.parametrize("shared", [1, 0])
@pytest.mark.parametrize("k,r,L,G,erase", [(196, 59, 9000, 6, None), (196, 59, 9000, 6, 3), (160, 48, 4100, 9, 40),
                                           (128, 39, 2100, 12, None), (128, 20, 9000, 6, None), (128, 20, 2100, 9, 20)])
def test_decode_c5_synw_shared(qf, oracle, gpu_ctx, k, r, L, G, erase, shared, monkeypatch):
    """Long-row C5 decode with the FFT syndrome passes item-major, their waves
    sharing the row gather through LDS ('Z', QF_OPT_SYNW_SHARED = 1), and
    pass-major ('Y' / plain 'X', 0): bit-exact either way, with few erasures
    (most items then skip the upper passes but still produce their share of
    the rows) and with many, and a partial last unit (L % 16 != 0)."""
    _path(monkeypatch, "default_1wave")
    qf.set_default_options(synw_shared=shared)
    rng = np.random.default_rng(k * 31 + L + (erase or 0))
    kw = {"erase": erase, "shuffle": False} if erase is not None else {}
    max_rows = k + r
    src, gens = make_batch(oracle, rng, k, r, L, G, max_rows, **kw)
    out = run_decode(qf, k, r, L, G, max_rows, gens, False)
    check(oracle, k, L, src, gens, out, False)
