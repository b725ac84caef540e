"""The generated bit-sliced Cauchy kernel, executed by the IR emulator on
CPU against the oracle: results, memory bounds and load/wait discipline.
(The same IR is emitted as gfx950 assembly; tests/test_gpu_encode.py runs
the assembled kernel on the device.)"""
import numpy as np
import pytest

from quicfuscate_amd import bs_codegen as bs


@pytest.mark.parametrize("k,r,pd,L,G,waves", [
    (8, 4, 2, 96, 5, 2),     # whole 32-byte chunks
    (8, 4, 2, 80, 7, 3),     # L % 32 == 16: a half chunk per row
    (5, 3, 3, 64, 4, 1),     # odd k, prefetch deeper than k
    (1, 1, 1, 64, 3, 1),
    (16, 16, 4, 1200, 3, 2), # a full-width accumulator set
    (64, 16, 3, 1200, 2, 1), # the benchmark kernel (units of two generations per lane)
])
def test_emulated_kernel_matches_oracle(oracle, k, r, pd, L, G, waves):
    spec = bs.KernelSpec(k, r, pd)
    ops = bs.generate(spec)
    rng = np.random.default_rng(k * 100 + r + L)
    srs = L + 16 * (k % 3)          # row stride > L on some shapes
    sgs = k * srs + 32
    drs = L + 32
    dgs = r * drs + 16
    src = rng.integers(0, 256, G * sgs, dtype=np.uint8)
    dst = np.full(G * dgs, 0xEE, np.uint8)
    emu = bs.Emulator(ops)
    SRC, DST = 0x10000000, 0x40000000
    emu.add_buffer(SRC, src)
    emu.add_buffer(DST, dst)
    ka = bs.kernargs(SRC, DST, sgs, dgs, srs, drs, L, G, waves * 4)
    for wg in range(waves):
        for w in range(4):
            emu.run_wave(ka, wg, w)
    for g in range(G):
        rows = np.stack([src[g * sgs + i * srs: g * sgs + i * srs + L] for i in range(k)])
        want = oracle.encode(rows, r)
        for j in range(r):
            off = g * dgs + j * drs
            assert (dst[off: off + L] == want[j]).all(), (g, j)
            assert (dst[off + L: off + drs] == 0xEE).all()


@pytest.mark.parametrize("k,r,L,G,zero_tail", [
    (8, 4, 80, 7, True),      # L = 5 units -> Lv = 8: three padding lanes per row
    (8, 4, 1200, 3, True),    # the benchmark row length: Lv = 80
    (5, 3, 96, 9, False),     # padded lane space without tail writes
    (64, 16, 1200, 2, True),
])
def test_emulated_kernel_padded_lanes(oracle, k, r, L, G, zero_tail):
    """Lane space of Lv = round_up(L/16, 8) units per row: padding lanes load
    nothing; with zero_tail they write zeros to [L, 16 Lv) of every repair
    row, and never past it."""
    spec = bs.KernelSpec(k, r, 3)
    ops = bs.generate(spec)
    Lv = bs.padded_units(L)
    rng = np.random.default_rng(k + 3 * L + G)
    srs = L + 16 * (k % 2)
    sgs = k * srs
    drs = 16 * Lv + 128
    dgs = r * drs
    src = rng.integers(0, 256, G * sgs, dtype=np.uint8)
    dst = np.full(G * dgs, 0xEE, np.uint8)
    emu = bs.Emulator(ops)
    SRC, DST = 0x10000000, 0x40000000
    emu.add_buffer(SRC, src)
    emu.add_buffer(DST, dst)
    _, _, items = bs.launch_geometry(L, G, Lv)
    waves = (items + 3) // 4
    ka = bs.kernargs(SRC, DST, sgs, dgs, srs, drs, L, G, waves * 4, Lv=Lv, zero_tail=zero_tail)
    for wg in range(waves):
        for w in range(4):
            emu.run_wave(ka, wg, w)
    for g in range(G):
        rows = np.stack([src[g * sgs + i * srs: g * sgs + i * srs + L] for i in range(k)])
        want = oracle.encode(rows, r)
        for j in range(r):
            off = g * dgs + j * drs
            assert (dst[off: off + L] == want[j]).all(), (g, j)
            tail = dst[off + L: off + 16 * Lv]
            assert (tail == (0 if zero_tail else 0xEE)).all(), (g, j)
            assert (dst[off + 16 * Lv: off + drs] == 0xEE).all()


def test_emulator_catches_missing_wait():
    spec = bs.KernelSpec(4, 2, 2)
    ops = [op for op in bs.generate(spec) if not (op.name == "s_waitcnt_vm" and op.args[0] == 2)]
    src = np.zeros(4 * 64 * 2, np.uint8)
    dst = np.zeros(2 * 64 * 2, np.uint8)
    emu = bs.Emulator(ops)
    emu.add_buffer(0x1000, src)
    emu.add_buffer(0x900000, dst)
    with pytest.raises(bs.EmuError):
        emu.run_wave(bs.kernargs(0x1000, 0x900000, 256, 128, 64, 64, 64, 2, 4), 0, 0)


def test_magic_division():
    for U in (2, 3, 5, 37, 38, 64, 100, 282, 1000):
        m, sh = bs.magic_for(U)
        for f in list(range(0, 5000)) + [2**22 + 17, 2**24 - 1, 2**30 + 12345]:
            assert ((f * m) >> 32) >> sh == f // U


def test_mul_matrix_rows_reproduce_field():
    for c in range(256):
        rows = bs.mul_matrix_rows(c)
        for x in (1, 2, 3, 0x53, 0x80, 0xFF):
            y = 0
            for b in range(8):
                y |= (bin(rows[b] & x).count("1") & 1) << b
            assert y == bs.gf_mul(c, x)


def _gf_matvec(D, rows):
    """sum_a D[b][a] * rows[a] over GF(256) (rows: e x L uint8)."""
    out = np.zeros((len(D), rows.shape[1]), np.uint8)
    for b, Db in enumerate(D):
        for a, c in enumerate(Db):
            out[b] ^= np.array([bs.gf_mul(c, int(x)) for x in range(256)], np.uint8)[rows[a]]
    return out


@pytest.mark.parametrize("k,r,pd,L,G,waves", [
    (8, 4, 2, 96, 6, 2),
    (8, 4, 3, 80, 7, 2),      # half chunks
    (16, 16, 4, 64, 5, 1),
    (5, 3, 1, 64, 9, 1),
    (8, 4, 3, 72, 5, 2),      # partial last unit (padded lane space only)
    (6, 5, 3, 41, 7, 1),
])
@pytest.mark.parametrize("padded", [False, True])
def test_emulated_syndrome_kernel(oracle, k, r, pd, L, G, waves, padded):
    """Decode stage A on the emulator: syndromes of the accepted repairs, and
    the closed-form Cauchy inverse applied to them gives the erased sources.
    With L % 16 != 0 the last unit is read whole (bytes past L are junk in
    the syndrome rows; the combine stores only L bytes)."""
    if L % 16 and not padded:
        pytest.skip("a partial last unit needs the padded lane space")
    spec = bs.KernelSpec(k, r, pd, mode="syn")
    ops = bs.generate(spec)
    rng = np.random.default_rng(7 * k + r + L)
    rs = L + 16
    n_slots = k + 2
    rgs = n_slots * rs + 16
    Lv = bs.padded_units(L) if padded else None
    srs = (16 * Lv if padded else L) + 32
    sgs = r * srs
    mstride = spec.map_stride
    rows = rng.integers(0, 256, G * rgs, dtype=np.uint8)
    smap = np.full(G * mstride, 0xFF, np.uint8)
    syn = np.full(G * sgs, 0xEE, np.uint8)
    plans = []
    for g in range(G):
        src = rng.integers(0, 256, (k, L), dtype=np.uint8)
        rep = oracle.encode(src, r)
        e = int(rng.integers(0, min(k, r) + 1))
        E = sorted(rng.choice(k, e, replace=False).tolist())
        J = rng.choice(r, e, replace=False).tolist()
        present = [("s", i) for i in range(k) if i not in E] + [("p", j) for j in J]
        order = rng.permutation(len(present))
        slots = rng.choice(n_slots, len(present), replace=False)  # spare slots stay junk
        for n, pi in enumerate(order):
            kind, idx = present[pi]
            sl = int(slots[n])
            data = src[idx] if kind == "s" else rep[idx]
            rows[g * rgs + sl * rs: g * rgs + sl * rs + L] = data
            smap[g * mstride + (idx if kind == "s" else k + idx)] = sl
        plans.append((src, rep, E, J))
    emu = bs.Emulator(ops)
    ROWS, SYN, MAP, ZERO = 0x10000000, 0x40000000, 0x70000000, 0x78000000
    emu.add_buffer(ROWS, rows)
    emu.add_buffer(SYN, syn)
    emu.add_buffer(MAP, smap)
    emu.add_buffer(ZERO, np.zeros((L + 15) // 16 * 16, np.uint8))
    ka = bs.kernargs(ROWS, SYN, rgs, sgs, rs, srs, L, G, waves * 4, smap=MAP, map_stride=mstride, zero=ZERO,
                     Lv=Lv)
    waves = max(waves, (bs.launch_geometry(L, G, Lv)[2] + 3) // 4)
    for wg in range(waves):
        for w in range(4):
            emu.run_wave(ka, wg, w)
    C = np.array(bs.cauchy(k, r), np.uint8)
    for g, (src, rep, E, J) in enumerate(plans):
        got = {}
        for j in range(r):
            blk = syn[g * sgs + j * srs: g * sgs + (j + 1) * srs]
            if j not in J:
                assert (blk == 0xEE).all(), (g, j)
                continue
            assert (blk[(16 * Lv if padded else L):] == 0xEE).all()
            want = rep[j].copy()
            for i in range(k):
                if i not in E:
                    want ^= np.array([bs.gf_mul(int(C[j, i]), x) for x in range(256)], np.uint8)[src[i]]
            assert (blk[:L] == want).all(), (g, j)
            got[j] = blk[:L]
        if E:
            D = bs.cauchy_inverse(k, J, E)
            rec = _gf_matvec(D, np.stack([got[j] for j in J]))
            assert (rec == src[E]).all(), g


def test_cauchy_inverse_closed_form():
    rng = np.random.default_rng(3)
    for _ in range(60):
        k = int(rng.integers(1, 200))
        r = int(rng.integers(1, min(40, 256 - k) + 1))
        e = int(rng.integers(1, min(k, r) + 1))
        E = sorted(rng.choice(k, e, replace=False).tolist())
        J = rng.choice(r, e, replace=False).tolist()
        C = [[bs.gf_inv(((k + j) & 255) ^ i) for i in E] for j in J]
        D = bs.cauchy_inverse(k, J, E)
        for b in range(e):
            for c in range(e):
                acc = 0
                for a in range(e):
                    acc ^= bs.gf_mul(D[b][a], C[a][c])
                assert acc == (1 if b == c else 0)


@pytest.mark.parametrize("k,r,mode", [(64, 16, "enc"), (64, 16, "syn"), (16, 1, "syn"), (32, 16, "enc"),
                                      (64, 16, "dec"), (16, 1, "dec"), (128, 20, "synw")])
def test_declared_register_budget_covers_code(k, r, mode):
    """Every VGPR / SGPR the generated code names lies below the
    .amdhsa_next_free_* counts of its kernel descriptor."""
    import re

    spec = bs.KernelSpec(k, r, 4, mode)
    text = bs.emit_asm(spec, bs.generate(spec))
    body, desc = text.split(".amdhsa_kernel", 1)
    nv = int(re.search(r"\.amdhsa_next_free_vgpr (\d+)", desc).group(1))
    ns = int(re.search(r"\.amdhsa_next_free_sgpr (\d+)", desc).group(1))
    vmax = smax = 0
    for m in re.finditer(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b", body):
        vmax = max(vmax, int(m.group(2) or m.group(3)))
    for m in re.finditer(r"\bs\[(\d+):(\d+)\]|\bs(\d+)\b", body):
        smax = max(smax, int(m.group(2) or m.group(3)))
    assert vmax < nv, (vmax, nv)
    assert smax < ns, (smax, ns)


@pytest.mark.parametrize("mode", ["enc", "syn"])
def test_xor3_variant_matches_plain(oracle, mode):
    """The v_bitop3 accumulate variant computes the same repairs/syndromes."""
    k, r, L, G = 8, 4, 80, 5
    rng = np.random.default_rng(17)
    outs = []
    for x3 in (False, True):
        spec = bs.KernelSpec(k, r, 2, mode, xor3=x3)
        emu = bs.Emulator(bs.generate(spec))
        src = rng.integers(0, 256, G * k * L, dtype=np.uint8) if not outs else outs[0][0]
        dst = np.zeros(G * r * L, np.uint8)
        emu.add_buffer(0x1000000, src)
        emu.add_buffer(0x9000000, dst)
        if mode == "enc":
            ka = bs.kernargs(0x1000000, 0x9000000, k * L, r * L, L, L, L, G, 4)
        else:
            smap = np.full(G * spec.map_stride, 0xFF, np.uint8)
            for g in range(G):
                smap[g * spec.map_stride: g * spec.map_stride + k] = np.arange(k)
                smap[g * spec.map_stride + k: g * spec.map_stride + k + 2] = [0, 1]  # repairs 0,1 at slots 0,1
            emu.add_buffer(0x5000000, smap)
            emu.add_buffer(0x6000000, np.zeros(L, np.uint8))
            ka = bs.kernargs(0x1000000, 0x9000000, k * L, r * L, L, L, L, G, 4, smap=0x5000000,
                             map_stride=spec.map_stride, zero=0x6000000)
        emu.run_wave(ka, 0, 0)
        emu.run_wave(ka, 0, 1)
        emu.run_wave(ka, 0, 2)
        emu.run_wave(ka, 0, 3)
        outs.append((src, dst.copy()))
    assert (outs[0][1] == outs[1][1]).all()
    assert outs[0][1].any()


def test_xcd_remap_is_a_bijection():
    for nwg in range(1, 400):
        q, rem = nwg // 8, nwg % 8
        got = sorted((w % 8) * q + min(w % 8, rem) + w // 8 for w in range(nwg))
        assert got == list(range(nwg))


def _dec_case(oracle, k, r, pd, L, G, seed, erase=None, padded=True, chunked=False, offs=False,
              wave_gen=False, **spec_kw):
    """Run the fused decode kernel (mode "dec") on the emulator: random
    erasures (or `erase` sources), random accepted repairs in random slots,
    LU records from bs.lu_record; returns the number of wrong rows."""
    spec = bs.KernelSpec(k, r, pd, mode="dec", chunked=chunked, wave_gen=wave_gen,
                         **{a: b for a, b in spec_kw.items() if not a.startswith("_")})
    rng = np.random.default_rng(seed)
    rs = L + 16
    n_slots = k + 2
    rgs = n_slots * rs + 16
    Lv = bs.padded_units(L) if padded else None
    rrs = L + 32
    emax = min(k, r)
    ogs = emax * rrs + 16
    ms = spec.map_stride
    rows = rng.integers(0, 256, G * rgs, dtype=np.uint8)
    smap = np.full(G * ms, 0xFF, np.uint8)
    recs = np.zeros(G * bs.LU_REC_BYTES, np.uint8)
    out = np.full(G * ogs, 0xEE, np.uint8)
    plans = []
    for g in range(G):
        src = rng.integers(0, 256, (k, L), dtype=np.uint8)
        rep = oracle.encode(src, r)
        e = int(rng.integers(0, emax + 1)) if erase is None else erase
        E = sorted(rng.choice(k, e, replace=False).tolist())
        J = rng.choice(r, e, replace=False).tolist()
        present = [("s", i) for i in range(k) if i not in E] + [("p", j) for j in J]
        slots = rng.choice(n_slots, len(present), replace=False)
        for n, pi in enumerate(rng.permutation(len(present))):
            kind, idx = present[pi]
            sl = int(slots[n])
            rows[g * rgs + sl * rs: g * rgs + sl * rs + L] = src[idx] if kind == "s" else rep[idx]
            smap[g * ms + (idx if kind == "s" else k + idx)] = sl
        recs[g * bs.LU_REC_BYTES:(g + 1) * bs.LU_REC_BYTES] = bs.lu_record(k, r, J, E)
        plans.append((src, E))
    emu = bs.Emulator(bs.generate(spec))
    ROWS, OUT, MAP, ZERO, REC, TAB = 0x10000000, 0x40000000, 0x70000000, 0x78000000, 0x7C000000, 0x7E000000
    for base, buf in ((ROWS, rows), (OUT, out), (MAP, smap), (ZERO, np.zeros((L + 15) // 16 * 16, np.uint8)), (REC, recs),
                      (TAB, bs.split_tables())):
        emu.add_buffer(base, buf)
    if chunked:   # (L % 16 != 0: any Lv >= Lu gets past launch_geometry; chunked sets its own)
        Lv = (L + 15) // 16 if L % 16 else None
        items = G if wave_gen else (G * (((L + 15) // 16 + 1) // 2) + 63) // 64
        waves = (items + 3) // 4
        if spec.ksplit > 1:   # one workgroup per item (fewer: persistent)
            waves = max(1, items - spec_kw.get("_fewer_wgs", 0))
    else:
        waves = (bs.launch_geometry(L, G, Lv)[2] + 3) // 4
    so = do = 0
    gs_r, gs_o = rgs, ogs
    if offs:   # generation offset tables: generation g placed at reversed block positions
        T1, T2 = 0x7F000000, 0x7F800000
        emu.add_buffer(T1, np.array([(G - 1 - g) * rgs for g in range(G)], np.uint64).view(np.uint8))
        emu.add_buffer(T2, np.array([(G - 1 - g) * ogs for g in range(G)], np.uint64).view(np.uint8))
        so, do, gs_r, gs_o = T1, T2, 0, 0
        rows_l = rows.reshape(G, rgs)[::-1].copy().reshape(-1)
        emu.mem[ROWS][:] = rows_l
    ka = bs.kernargs(ROWS, OUT, gs_r, gs_o, rs, rrs, L, G, waves * 4, smap=MAP, map_stride=ms, zero=ZERO,
                     Lv=Lv, lu=(REC, bs.LU_REC_BYTES), tables=TAB, src_offs=so, dst_offs=do, chunked=chunked,
                     wave_gen=wave_gen)
    for wg in range(waves):
        if spec.ksplit > 1:
            emu.run_workgroup(ka, wg, 4, spec.lds_bytes)
            continue
        for w in range(4):
            emu.run_wave(ka, wg, w)
    if offs:
        out[:] = out.reshape(G, ogs)[::-1].copy().reshape(-1)
    bad = 0
    for g, (src, E) in enumerate(plans):
        blk = out[g * ogs: (g + 1) * ogs]
        for b, i in enumerate(E):
            bad += int(not (blk[b * rrs: b * rrs + L] == src[i]).all())
            assert (blk[b * rrs + L: (b + 1) * rrs] == 0xEE).all(), "bytes past L written"
        assert (blk[len(E) * rrs:] == 0xEE).all(), "rows past e written"
    return bad


@pytest.mark.parametrize("k,r,pd,L,G,seed,erase", [
    (8, 4, 2, 96, 6, 1, None),
    (8, 4, 3, 80, 7, 2, None),      # half chunks, padded lane space
    (16, 16, 4, 64, 5, 3, None),    # every block can be a pivot
    (16, 16, 2, 96, 4, 4, 16),      # e = r: all 16 blocks, jmax = 16
    (5, 3, 1, 64, 9, 5, 0),         # nothing erased: no stores at all
])
def test_emulated_fused_decode(oracle, k, r, pd, L, G, seed, erase):
    """Fused decode on the emulator: syndromes, in-register LU solve with the
    split tables from LDS, recovered rows equal the erased sources."""
    assert _dec_case(oracle, k, r, pd, L, G, seed, erase) == 0


def test_lu_record_reconstructs_cauchy_submatrix():
    """The packed LU record's factors multiply back to C[J, E] (J ascending)."""
    rng = np.random.default_rng(11)
    for _ in range(40):
        k = int(rng.integers(1, 240))
        r = int(rng.integers(1, min(16, 256 - k) + 1))
        e = int(rng.integers(1, min(k, r) + 1))
        E = sorted(rng.choice(k, e, replace=False).tolist())
        J = rng.choice(r, e, replace=False).tolist()
        rec = bs.lu_record(k, r, J, E)
        Js = sorted(J)
        for t in range(16):
            assert rec[256 + t] == (Js.index(t) if t in Js else 0xFF)
        Lm = [[1 if b == c else (rec[16 * Js[c] + Js[b]] if b > c else 0) for c in range(e)] for b in range(e)]
        piv = [bs.gf_inv(rec[16 * Js[b] + Js[b]]) for b in range(e)]    # U[b][b]
        Um = [[(piv[b] if b == c else bs.gf_mul(rec[16 * Js[c] + Js[b]], piv[b])) if b <= c else 0
               for c in range(e)] for b in range(e)]
        for b in range(e):
            for c in range(e):
                acc = 0
                for q in range(e):
                    acc ^= bs.gf_mul(Lm[b][q], Um[q][c])
                assert acc == bs.gf_inv(((k + Js[b]) & 0xFF) ^ E[c])


def test_emulated_fused_decode_unpadded_lanes(oracle):
    """The library launches the fused decode over the unpadded lane space
    (L/16 units per row): halves of a lane straddle generations."""
    assert _dec_case(oracle, 8, 4, 2, 80, 9, 6, None, padded=False) == 0
    assert _dec_case(oracle, 16, 16, 3, 1200, 2, 7, 13, padded=False) == 0


@pytest.mark.parametrize("k,rt,L,G,split,fewer", [
    (8, 4, 72, 5, 4, 0),       # L % 16 = 8: partial last unit, one pass
    (6, 5, 100, 4, 3, 0),      # passes of 3 + 2 repairs
    (9, 20, 1200, 3, 16, 0),   # passes of 16 + 4, the C2 row length
    (4, 3, 64, 40, 3, 2),      # k = ks, 3 items on one workgroup (persistent loop)
])
def test_emulated_encode_ksplit(oracle, k, rt, L, G, split, fewer):
    """ksplit = 4 encode (qf_cauchy_bss_*): the four waves of a workgroup take
    sources w, w + 4, ... of one item and wave 0 sums the partial repairs
    through LDS (barriers emulated) before the zero-tail stores."""
    Lv = bs.padded_units(L)
    rng = np.random.default_rng(k * 37 + L + rt)
    srs = (L + 15) // 16 * 16 + 16 * (k % 2)
    sgs = k * srs
    drs = 16 * Lv + 64
    dgs = rt * drs
    src = rng.integers(0, 256, G * sgs, dtype=np.uint8)
    dst = np.full(G * dgs, 0xEE, np.uint8)
    SRC, DST = 0x10000000, 0x40000000
    _, _, items = bs.launch_geometry(L, G, Lv)
    wgs = max(1, items - fewer)
    for j0 in range(0, rt, split):
        spec = bs.KernelSpec(k, min(split, rt - j0), 3, r_total=rt, j0=j0, ksplit=4)
        emu = bs.Emulator(bs.generate(spec))
        emu.add_buffer(SRC, src)
        emu.add_buffer(DST, dst)
        ka = bs.kernargs(SRC, DST + j0 * drs, sgs, dgs, srs, drs, L, G, wgs * 4, Lv=Lv, zero_tail=True)
        for wg in range(wgs):
            emu.run_workgroup(ka, wg, 4, spec.lds_bytes)
    for g in range(G):
        rows = np.stack([src[g * sgs + i * srs: g * sgs + i * srs + L] for i in range(k)])
        want = oracle.encode(rows, rt)
        for j in range(rt):
            off = g * dgs + j * drs
            assert (dst[off: off + L] == want[j]).all(), (g, j)
            assert (dst[off + L: off + 16 * Lv] == 0).all(), (g, j)
            assert (dst[off + 16 * Lv: off + drs] == 0xEE).all()


@pytest.mark.parametrize("k,rt,L,G,split", [
    (8, 4, 72, 5, 4),      # L % 16 = 8: partial last unit, one pass
    (6, 5, 100, 4, 3),     # L % 16 = 4, passes of 3 + 2 repairs
    (5, 7, 33, 6, 4),      # one byte in the last unit, passes of 4 + 3
    (4, 20, 64, 3, 16),    # whole units, passes of 16 + 4
])
def test_emulated_kernel_tail_and_passes(oracle, k, rt, L, G, split):
    """Zero-tail lane space with a partial last unit (its bytes >= L, read from
    the source rows' padding, are masked to zero) and codes split into
    passes of repairs j0.. (each pass writes its own repair rows)."""
    Lv = bs.padded_units(L)
    rng = np.random.default_rng(k * 31 + L + rt)
    srs = (L + 15) // 16 * 16 + 16 * (k % 2)
    sgs = k * srs
    drs = 16 * Lv + 64
    dgs = rt * drs
    src = rng.integers(0, 256, G * sgs, dtype=np.uint8)   # padding bytes are garbage too
    dst = np.full(G * dgs, 0xEE, np.uint8)
    SRC, DST = 0x10000000, 0x40000000
    _, _, items = bs.launch_geometry(L, G, Lv)
    waves = (items + 3) // 4
    for j0 in range(0, rt, split):
        spec = bs.KernelSpec(k, min(split, rt - j0), 3, r_total=rt, j0=j0)
        emu = bs.Emulator(bs.generate(spec))
        emu.add_buffer(SRC, src)
        emu.add_buffer(DST, dst)
        ka = bs.kernargs(SRC, DST + j0 * drs, sgs, dgs, srs, drs, L, G, waves * 4, Lv=Lv, zero_tail=True)
        for wg in range(waves):
            for w in range(4):
                emu.run_wave(ka, wg, w)
    for g in range(G):
        rows = np.stack([src[g * sgs + i * srs: g * sgs + i * srs + L] for i in range(k)])
        want = oracle.encode(rows, rt)
        for j in range(rt):
            off = g * dgs + j * drs
            assert (dst[off: off + L] == want[j]).all(), (g, j)
            assert (dst[off + L: off + 16 * Lv] == 0).all(), (g, j)
            assert (dst[off + 16 * Lv: off + drs] == 0xEE).all()


def test_tail_masks():
    assert bs.tail_masks(64) == [0xFFFFFFFF] * 4
    assert bs.tail_masks(72) == [0xFFFFFFFF, 0xFFFFFFFF, 0, 0]
    assert bs.tail_masks(33) == [0xFF, 0, 0, 0]
    assert bs.tail_masks(9000) == [0xFFFFFFFF, 0xFFFFFFFF, 0, 0]
    assert bs.tail_masks(46) == [0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFF]


def test_register_budget_large_pass_kernel():
    """A C5 pass kernel (k = 196, repairs 16..31 of r = 59) is past the
    s_branch range: far jumps through s[66:67], within its declared SGPRs."""
    import re

    spec = bs.KernelSpec(196, 16, 3, "enc", r_total=59, j0=16)
    assert spec.far and spec.name == "qf_cauchy_bs_k196_r59_j16"
    text = bs.emit_asm(spec, bs.generate(spec))
    body, desc = text.split(".amdhsa_kernel", 1)
    ns = int(re.search(r"\.amdhsa_next_free_sgpr (\d+)", desc).group(1))
    nv = int(re.search(r"\.amdhsa_next_free_vgpr (\d+)", desc).group(1))
    smax = max(int(m.group(2) or m.group(3)) for m in re.finditer(r"\bs\[(\d+):(\d+)\]|\bs(\d+)\b", body))
    vmax = max(int(m.group(2) or m.group(3)) for m in re.finditer(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b", body))
    assert smax < ns and vmax < nv, (smax, ns, vmax, nv)
    assert "s_setpc_b64 s[66:67]" in body


def test_emulated_offset_tables_encode(oracle):
    """Generation offset tables (the heterogeneous batch API): generation g's
    rows start at base + table[g] (any order, any gaps) instead of
    base + g * gen_stride; encode and fused decode both honour them."""
    k, r, L, G = 8, 4, 96, 5
    rng = np.random.default_rng(44)
    srs = L
    blk = k * srs
    perm = rng.permutation(G)
    src_off = np.array([int(p) * (blk + 48) + 16 for p in perm], np.uint64)       # shuffled, gapped
    rep_off = np.array([int(p) * (r * L + 32) for p in rng.permutation(G)], np.uint64)
    src = rng.integers(0, 256, G * (blk + 48) + 64, dtype=np.uint8)
    dst = np.full(G * (r * L + 32) + 64, 0xEE, np.uint8)
    spec = bs.KernelSpec(k, r, 2)
    emu = bs.Emulator(bs.generate(spec))
    SRC, DST, T1, T2 = 0x10000000, 0x40000000, 0x60000000, 0x61000000
    emu.add_buffer(SRC, src)
    emu.add_buffer(DST, dst)
    emu.add_buffer(T1, src_off.view(np.uint8))
    emu.add_buffer(T2, rep_off.view(np.uint8))
    ka = bs.kernargs(SRC, DST, 0, 0, srs, L, L, G, 8, src_offs=T1, dst_offs=T2)
    for wg in range(2):
        for w in range(4):
            emu.run_wave(ka, wg, w)
    for g in range(G):
        so, ro = int(src_off[g]), int(rep_off[g])
        rows = np.stack([src[so + i * srs: so + i * srs + L] for i in range(k)])
        want = oracle.encode(rows, r)
        for j in range(r):
            assert (dst[ro + j * L: ro + (j + 1) * L] == want[j]).all(), (g, j)


@pytest.mark.parametrize("k,r,pd,L,G,seed,erase,offs", [
    (8, 4, 2, 96, 6, 1, None, False),
    (8, 4, 3, 80, 7, 2, None, False),     # Lu = 5: Q = 3, the last lane-chunk has no B unit
    (16, 16, 4, 64, 5, 3, None, True),    # offset tables
    (16, 16, 2, 96, 4, 4, 16, False),     # e = r: all 16 blocks
    (5, 3, 1, 64, 9, 5, 0, False),        # nothing erased
    (16, 16, 3, 1200, 2, 7, 13, True),    # the C3 row length (Q = 38: lane-chunks straddle items)
    (8, 5, 2, 100, 5, 8, None, False),    # L % 16 = 4: the tail lane stores its unit B bytewise
    (16, 10, 3, 9000, 1, 9, 6, False),    # the C5 jumbo length (Lu = 563, L % 16 = 8)
    (8, 4, 2, 47, 6, 10, None, True),     # Lu = 3, L % 16 = 15, offset tables
])
def test_emulated_fused_decode_chunked(oracle, k, r, pd, L, G, seed, erase, offs):
    """The lane-chunk fused decode (one generation per lane: units q and
    q + Q) recovers the erased sources, with strided generations or offset
    tables, and writes nothing else."""
    assert _dec_case(oracle, k, r, pd, L, G, seed, erase, padded=False, chunked=True, offs=offs) == 0


@pytest.mark.parametrize("lu_ilp", [False, True])
@pytest.mark.parametrize("k,r,pd,L,G,seed,erase", [
    (16, 16, 2, 96, 4, 4, 16),            # all 16 blocks
    (16, 16, 3, 1200, 2, 7, 13),
    (8, 5, 2, 100, 5, 8, None),
])
def test_emulated_fused_decode_lu_schedule(oracle, k, r, pd, L, G, seed, erase, lu_ilp):
    """The interleaved LU schedule (lu_ilp: 2-3 dwords' products in separate
    temps, selectors stage by stage) recovers the same rows."""
    assert _dec_case(oracle, k, r, pd, L, G, seed, erase, padded=False, chunked=True, lu_ilp=lu_ilp) == 0


@pytest.mark.parametrize("k,r,pd,L,G,seed,erase,offs,fewer", [
    (8, 4, 2, 96, 6, 1, None, False, 0),
    (16, 16, 3, 1200, 2, 7, 13, False, 0),   # lane-chunks straddle items; jmax up to 16
    (16, 16, 2, 96, 4, 4, 16, True, 0),      # all 16 blocks, offset tables
    (5, 3, 1, 64, 9, 5, 0, False, 0),        # nothing erased
    (8, 5, 2, 100, 5, 8, None, False, 0),    # L % 16 = 4: bytewise tail
    (3, 4, 2, 64, 5, 11, None, False, 0),    # k < 4: a wave with no source row
    (16, 10, 3, 1200, 6, 12, 6, False, 2),   # fewer workgroups than items: persistent loop
])
def test_emulated_fused_decode_ksplit(oracle, k, r, pd, L, G, seed, erase, offs, fewer):
    """ksplit = 4 (qf_cauchy_decs_*): the four waves of a workgroup split an
    item's rows, waves 1..3 hand partial syndromes to wave 0 through LDS
    (barriers emulated), and the recovered rows equal the sources."""
    assert _dec_case(oracle, k, r, pd, L, G, seed, erase, padded=False, chunked=True, offs=offs, ksplit=4,
                     _fewer_wgs=fewer) == 0


@pytest.mark.parametrize("k,r,pd,L,G,seed,erase", [
    (8, 4, 2, 96, 6, 1, None),
    (16, 16, 3, 1200, 2, 7, 13),
])
def test_emulated_fused_decode_wave_gen(oracle, k, r, pd, L, G, seed, erase):
    """Lab variant (tools/dec_lab.py): one generation per wave, erased source
    rows skipped by a wave-uniform branch; same recovered rows."""
    assert _dec_case(oracle, k, r, pd, L, G, seed, erase, padded=False, chunked=True, wave_gen=True) == 0


@pytest.mark.parametrize("k,r,mode,chunked", [(64, 16, "enc", False), (64, 16, "syn", False),
                                               (64, 16, "dec", False), (64, 16, "dec", True),
                                               (16, 1, "dec", True), (96, 15, "dec", True),
                                               (128, 20, "synw", False)])
def test_register_tuples_even_aligned(k, r, mode, chunked):
    """gfx950 requires every multi-register VGPR operand (v[a:b]) to start at
    an even register; the assembler rejects odd tuples.  Checked on the IR's
    assembly text here so it fails on CPU, not at build time on the box."""
    import re

    spec = bs.KernelSpec(k, r, 3, mode, chunked=chunked)
    body = bs.emit_asm(spec, bs.generate(spec)).split(".amdhsa_kernel", 1)[0]
    odd = {m.group(0) for m in re.finditer(r"\bv\[(\d+):(\d+)\]", body) if int(m.group(1)) % 2}
    assert not odd, sorted(odd)[:5]
    if chunked:
        nv = spec.next_free_vgpr
        assert nv <= 256


def _synw_case(oracle, k, rt, rp, L, G, seed, offs=False, use_bound=True, merged=False, fft=0, concat=False,
               xchg=False, helpers=0, xchg_early=0):
    """The wave-uniform syndrome kernel (mode "synw") on the emulator for
    every pass j0 of (k, rt) in steps of rp: accepted repairs' syndromes of
    generations with a repair >= j0 equal p_j ^ C[j, S] x_S; items whose
    generations' bound <= j0 are skipped."""
    rng = np.random.default_rng(seed)
    rs = L + 48
    n_slots = k + rt
    rgs = n_slots * rs + 32
    Lv = bs.padded_units(L)
    srs = 16 * Lv + 16
    sgs = rt * srs
    if fft:   # additive-FFT passes: one per coset of 16 repair points (lch_fft.coset_passes)
        from quicfuscate_amd import lch_fft

        specs = [bs.KernelSpec(k, n, 2, mode="synw", r_total=rt, j0=j0, fft=fft, xchg_early=xchg_early)
                 for j0, n in lch_fft.coset_passes(k, rt)]
    else:
        specs = [bs.KernelSpec(k, min(rp, rt - j0), 2, mode="synw", r_total=rt, j0=j0) for j0 in range(0, rt, rp)]
    ms = specs[0].map_stride
    rows = rng.integers(0, 256, G * rgs + 4096, dtype=np.uint8)
    smap = np.full(G * ms, 0xFF, np.uint8)
    syn = np.full(G * sgs, 0xEE, np.uint8)
    bound = np.zeros(G, np.uint32)
    gen_off = rng.permutation(G) * rgs if offs else np.arange(G) * rgs   # rows of g at gen_off[g]
    plans = []
    for g in range(G):
        src = rng.integers(0, 256, (k, L), dtype=np.uint8)
        rep = oracle.encode(src, rt)
        e = int(rng.integers(0, min(k, rt) + 1)) if g % 3 else 0      # every third: nothing lost
        E = sorted(rng.choice(k, e, replace=False).tolist())
        J = sorted(rng.choice(rt, e, replace=False).tolist())
        present = [("s", i) for i in range(k) if i not in E] + [("p", j) for j in J]
        slots = rng.choice(n_slots, len(present), replace=False)
        for n, (kind, idx) in enumerate(present):
            sl = int(slots[n])
            data = src[idx] if kind == "s" else rep[idx]
            o = int(gen_off[g]) + sl * rs
            rows[o: o + L] = data
            smap[g * ms + (idx if kind == "s" else k + idx)] = sl
        bound[g] = (max(J) + 1) if J else 0
        plans.append((src, rep, E, J))
    emu_bufs = {}
    ROWS, SYN, MAP, ZERO, OFFS, BOUND = 0x10000000, 0x40000000, 0x70000000, 0x78000000, 0x7C000000, 0x7E000000
    # merged: every pass in one dispatch (MergedSpec), wave p of workgroup w
    # running pass p on item w
    for spec in ([bs.merged_spec(specs, concat, xchg=xchg, helpers=helpers)] if merged else specs):
        emu = bs.Emulator(bs.generate(spec))
        emu.add_buffer(ROWS, rows)
        emu.add_buffer(SYN, syn)
        emu.add_buffer(MAP, smap)
        emu.add_buffer(ZERO, np.zeros(16 * Lv, np.uint8))
        emu.add_buffer(OFFS, np.asarray(gen_off, np.uint64).view(np.uint8).copy())
        emu.add_buffer(BOUND, bound.view(np.uint8).copy())
        ka = bs.kernargs(ROWS, SYN + spec.j0 * srs, 0 if offs else rgs, sgs, rs, srs, L, G, 8, smap=MAP,
                         map_stride=ms, zero=ZERO, Lv=Lv, src_offs=OFFS if offs else 0,
                         bound=BOUND if use_bound else 0)
        n_items = bs.launch_geometry(L, G, Lv)[2]
        if merged and concat:   # pass-major: n 4-wave workgroups per pass
            n = (n_items + 3) // 4
            ka = bs.kernargs(ROWS, SYN, 0 if offs else rgs, sgs, rs, srs, L, G, 4 * n, smap=MAP,
                             map_stride=ms, zero=ZERO, Lv=Lv, src_offs=OFFS if offs else 0,
                             bound=BOUND if use_bound else 0)
            for wg in range(spec.n_passes * n):
                for w in range(4):
                    emu.run_wave(ka, wg, w)
            break
        if merged:
            ka = bs.kernargs(ROWS, SYN, 0 if offs else rgs, sgs, rs, srs, L, G, n_items, smap=MAP,
                             map_stride=ms, zero=ZERO, Lv=Lv, src_offs=OFFS if offs else 0,
                             bound=BOUND if use_bound else 0)
            for wg in range(n_items):
                if xchg:    # the waves share LDS and meet at barriers
                    emu.run_workgroup(ka, wg, spec.waves, spec.lds_bytes)
                    continue
                for w in range(spec.waves):
                    emu.run_wave(ka, wg, w)
            break
        for wv in range(n_items):
            emu.run_wave(ka, wv // 4, wv % 4)
        emu_bufs[spec.j0] = emu
    C = np.array(bs.cauchy(k, rt), np.uint8)
    mul = np.array([[bs.gf_mul(c, x) for x in range(256)] for c in range(256)], np.uint8)
    checked = 0
    for g, (src, rep, E, J) in enumerate(plans):
        for j in J:
            want = rep[j].copy()
            for i in range(k):
                if i not in E:
                    want ^= mul[C[j, i]][src[i]]
            blk = syn[g * sgs + j * srs: g * sgs + j * srs + L]
            assert (blk == want).all(), (g, j)
            checked += 1
    # skipped items: a generation (and its item neighbours) with bound <= j0 of
    # every pass it could have been processed in left its rows untouched
    if use_bound:
        for g in range(G):
            nb = [bound[x] for x in (g - 1, g, g + 1) if 0 <= x < G]
            for spec in specs:
                if max(nb) <= spec.j0:
                    blk = syn[g * sgs + spec.j0 * srs: g * sgs + (spec.j0 + spec.r) * srs]
                    assert (blk == 0xEE).all(), (g, spec.j0)
    return checked


@pytest.mark.parametrize("k,rt,rp,L,G,offs", [
    (8, 6, 3, 2048, 5, False),     # two passes, exact units
    (8, 6, 6, 2100, 4, False),     # one pass, partial last unit, padded lanes (Lv = 136: items straddle)
    (12, 7, 4, 2064, 4, True),     # generation offset table, uneven passes
    (5, 3, 2, 2200, 3, False),
])
def test_emulated_synw_kernel(oracle, k, rt, rp, L, G, offs):
    assert _synw_case(oracle, k, rt, rp, L, G, seed=k * 100 + rt + L, offs=offs) > 0


@pytest.mark.parametrize("concat", [False, True])
@pytest.mark.parametrize("k,rt,rp,L,G,offs", [(8, 6, 3, 2048, 5, False), (12, 7, 4, 2064, 4, True),
                                               (5, 3, 1, 2200, 3, False), (8, 6, 2, 4100, 9, False)])
def test_emulated_synw_merged(oracle, k, rt, rp, L, G, offs, concat):
    """All synw passes in one dispatch, item-major (a workgroup's waves run
    the passes on one item) or pass-major (concat: workgroup ranges per
    pass): the same syndromes, and the same skips, as one launch per pass."""
    assert _synw_case(oracle, k, rt, rp, L, G, seed=k * 100 + rt + L + 1, offs=offs, merged=True,
                      concat=concat) > 0


@pytest.mark.parametrize("k,rt,L,G,offs", [(24, 10, 2048, 3, False), (20, 20, 2100, 2, True), (48, 21, 2064, 2, False)])
def test_emulated_synw_fft(oracle, k, rt, L, G, offs):
    """synw passes through the hybrid additive FFT (lch_fft.hybrid_plan;
    absent sources read the zero row, accepted repairs XOR onto their
    transposed blocks): the same syndromes and skips as the plain passes."""
    assert _synw_case(oracle, k, rt, 0, L, G, seed=k * 7 + rt + L, offs=offs, fft=8) > 0


@pytest.mark.parametrize("early", [0, 5])
@pytest.mark.parametrize("k,rt,L,G,offs,helpers", [(24, 10, 2048, 3, False, 0), (20, 20, 2100, 4, True, 0),
                                                   (48, 21, 2064, 3, False, 0), (196, 59, 2048, 2, False, 0),
                                                   (48, 21, 2064, 3, True, 1), (20, 20, 2100, 4, False, 2),
                                                   (128, 20, 2048, 2, False, 0)])
def test_emulated_synw_xchg(oracle, k, rt, L, G, offs, helpers, early):
    """Item-major merged FFT synw whose waves share the source rows' gather,
    transposes and chunk butterflies through LDS (merged_spec(xchg=True)):
    the same syndromes and skips as the per-pass kernels; a skipped pass's
    wave still produces its groups (the barriers stay matched)."""
    assert _synw_case(oracle, k, rt, 0, L, G, seed=k * 11 + rt + L, offs=offs, fft=8, merged=True, xchg=True,
                      helpers=helpers, xchg_early=early) > 0


def test_emulated_synw_without_bound(oracle):
    assert _synw_case(oracle, 8, 5, 5, 2048, 3, seed=3, use_bound=False) > 0


def test_synw_register_budget():
    """The C5 shapes' synw passes fit 256 VGPRs (pd 3) and the SGPR budget."""
    for k, rt, rp in ((128, 20, 20), (160, 48, 16), (196, 59, 20), (128, 39, 20)):
        for j0 in range(0, rt, rp):
            spec = bs.KernelSpec(k, min(rp, rt - j0), 3, mode="synw", r_total=rt, j0=j0)
            assert spec.next_free_vgpr <= 256 and spec.next_free_sgpr <= 102


def test_transpose_shift64_equals_bfi():
    """The 64-bit-shift transpose network (stages 1-2 on register pairs) maps
    every 32-byte chunk to the same planes as the 32-bit one (and back)."""
    rng = np.random.default_rng(8)
    data = rng.integers(0, 1 << 32, (16, 64), dtype=np.uint64)
    end = [bs.Op("s_endpgm", ())]
    a = _run_regs(bs._transpose_ops(48, True) + bs._transpose_ops(56, True) + end, data)
    b = _run_regs(bs._transpose_ops(48, "s64") + bs._transpose_ops(56, "s64") + end, data)
    assert (a == b).all()
    twice = _run_regs(bs._transpose_ops(48, "s64") + bs._transpose_ops(48, "s64") + end, data)
    assert (twice[:8] == data[:8]).all()   # an involution


def _run_regs(ops, regs):
    """Execute straight-line transpose ops with v48..v63 preloaded; returns v48..v63."""
    v = np.zeros((256, 64), np.uint64)
    v[48:64] = regs
    s = [0] * 104
    s[bs.S_TMASK], s[bs.S_TMASK + 1], s[bs.S_TMASK + 2] = 0x0F0F0F0F, 0x33333333, 0x55555555
    M = np.uint64(0xFFFFFFFF)
    for op in ops:
        n, a = op.name, op.args
        if n == "v_lshl":
            v[a[0]] = (v[a[2]] << np.uint64(a[1])) & M
        elif n == "v_lshr":
            v[a[0]] = v[a[2]] >> np.uint64(a[1])
        elif n in ("v_lshl64", "v_lshr64"):
            x = v[a[2]] | (v[a[2] + 1] << np.uint64(32))
            x = (x << np.uint64(a[1])) if n == "v_lshl64" else (x >> np.uint64(a[1]))
            v[a[0]], v[a[0] + 1] = x & M, x >> np.uint64(32)
        elif n == "v_bitsel_s":
            m = np.uint64(s[a[1]])
            v[a[0]] = (m & v[a[2]]) | (~m & M & v[a[3]])
        elif n == "s_endpgm":
            break
        else:
            raise AssertionError(n)
    return v[48:64]


@pytest.mark.parametrize("mode", ["enc", "syn"])
def test_shift64_kernels_match_default(oracle, mode):
    """Whole kernels with the 64-bit-shift transposes compute the same bytes."""
    k, r, L, G = 8, 4, 96, 5
    rng = np.random.default_rng(23)
    outs = []
    for bfi in (True, "s64"):
        spec = bs.KernelSpec(k, r, 2, mode, bfi_transpose=bfi)
        emu = bs.Emulator(bs.generate(spec))
        src = rng.integers(0, 256, G * k * L, dtype=np.uint8) if not outs else outs[0][0]
        dst = np.zeros(G * r * L, np.uint8)
        emu.add_buffer(0x1000000, src)
        emu.add_buffer(0x9000000, dst)
        if mode == "enc":
            ka = bs.kernargs(0x1000000, 0x9000000, k * L, r * L, L, L, L, G, 4)
        else:
            smap = np.full(G * spec.map_stride, 0xFF, np.uint8)
            for g in range(G):
                smap[g * spec.map_stride: g * spec.map_stride + k] = np.arange(k)
                smap[g * spec.map_stride + k: g * spec.map_stride + k + 2] = [0, 1]
            emu.add_buffer(0x5000000, smap)
            emu.add_buffer(0x6000000, np.zeros(L, np.uint8))
            ka = bs.kernargs(0x1000000, 0x9000000, k * L, r * L, L, L, L, G, 4, smap=0x5000000,
                             map_stride=spec.map_stride, zero=0x6000000)
        for w in range(8):
            emu.run_wave(ka, w // 4, w % 4)
        outs.append((src, dst.copy()))
    assert (outs[0][1] == outs[1][1]).all() and outs[0][1].any()


def _gf_table():
    t = np.zeros((256, 256), np.uint8)
    for a in range(256):
        for b in range(256):
            t[a, b] = bs.gf_mul(a, b)
    return t


_GFT = None


def _cmb_case(L, G, seed, pas=0, offs=False, R=16, lean=False, pf2=False, jump=0):
    """qf_combine_bs on the emulator: out[j] = sum_{s < bound[g]} rec[g][s][j] *
    rows[g][s] for j < min(e[g] - 16 pass, R), bytes [0, L) only."""
    global _GFT
    if _GFT is None:
        _GFT = _gf_table()
    rng = np.random.default_rng(seed)
    spec = bs.KernelSpec(0, R, mode="cmb", cmb_lean=lean, cmb_pf2=pf2, cmb_jump=jump)
    Lp = (L + 15) // 16 * 16
    rs, drs = Lp + 32, Lp + 48
    nslot = 24
    rgs, dgs = nslot * rs + 16, 16 * drs + 32
    cgs = (nslot + 1) * 16
    rows = rng.integers(0, 256, G * rgs, dtype=np.uint8)
    rec = rng.integers(0, 256, G * cgs, dtype=np.uint8)
    e = rng.integers(16 * pas + 1, 16 * pas + R + 4, G).astype(np.uint32)
    bound = rng.integers(1, nslot + 1, G).astype(np.uint32)
    if G > 3:   # a generation without outputs in this pass, one without input rows
        e[1], bound[2] = 16 * pas, 0
    out = np.full(G * dgs, 0xEE, np.uint8)
    ROWS, OUT, REC, NO, BD, TAB, T1, T2 = (0x10000000, 0x40000000, 0x50000000, 0x60000000, 0x61000000,
                                           0x62000000, 0x63000000, 0x64000000)
    emu = bs.Emulator(bs.generate(spec))
    so = do = 0
    rgs_k, dgs_k = rgs, dgs
    if offs:   # generations at reversed block positions through offset tables
        emu.add_buffer(T1, np.array([(G - 1 - g) * rgs for g in range(G)], np.uint64).view(np.uint8))
        emu.add_buffer(T2, np.array([(G - 1 - g) * dgs for g in range(G)], np.uint64).view(np.uint8))
        so, do, rgs_k, dgs_k = T1, T2, 0, 0
    for base, buf in ((ROWS, rows), (OUT, out), (REC, rec), (NO, e), (BD, bound),
                      (TAB, bs.cmb_index_table().reshape(-1).view(np.uint8))):
        emu.add_buffer(base, buf.view(np.uint8))
    waves = 8
    ka, n_items = bs.cmb_kernargs(ROWS, OUT, rgs_k, dgs_k, rs, drs, REC, cgs, pas, NO, BD, TAB, L, G, waves,
                                  rows_offs=so, dst_offs=do)
    for w in range(waves):
        emu.run_wave(ka, w // 4, w % 4)
    bad = 0
    for g in range(G):
        gr = (G - 1 - g) if offs else g
        ew = int(min(max(int(e[g]) - 16 * pas, 0), R))
        blk = out[gr * dgs:(gr + 1) * dgs]
        for j in range(16):
            row = blk[j * drs:(j + 1) * drs]
            if j < ew:
                want = np.zeros(L, np.uint8)
                for sl in range(int(bound[g])):
                    c = rec[g * cgs + 16 * sl + j]
                    x = rows[gr * rgs + sl * rs: gr * rgs + sl * rs + L]
                    want ^= _GFT[c][x]
                bad += int(not (row[:L] == want).all())
                assert (row[L:] == 0xEE).all(), (g, j, "bytes past L written")
            else:
                assert (row == 0xEE).all(), (g, j, "row past ew written")
    return bad


@pytest.mark.parametrize("lean,pf2,jump", [(False, False, 0), (True, False, 0), (True, True, 0), (True, False, 3)])
@pytest.mark.parametrize("L,G,seed,pas,offs", [
    (64, 5, 1, 0, False),       # Lu = 4, Q = 2: one item per generation
    (100, 4, 2, 0, False),      # partial last unit (4 bytes)
    (1200, 2, 3, 1, True),      # second pass (outputs 16..), offset tables
    (4100, 2, 4, 0, False),     # Q = 129: three items per generation, tail of 4 bytes
    (33, 3, 5, 0, True),        # Lu = 3: unit B of lane 0 is the partial last unit
    (200, 9, 6, 0, False),      # e of every residue mod 4 (lean: products past e, never stored)
])
def test_emulated_combine_bs(L, G, seed, pas, offs, lean, pf2, jump):
    assert _cmb_case(L, G, seed, pas, offs, lean=lean, pf2=pf2, jump=jump) == 0


@pytest.mark.parametrize("lean,pf2,xcd,jump", [(False, False, False, 0), (True, False, False, 0), (True, True, False, 0),
                                               (True, False, True, 0), (True, False, True, 3), (True, False, False, 2)])
@pytest.mark.parametrize("L,G,P,offs", [(1200, 5, 3, False), (4100, 3, 2, True), (100, 9, 4, False)])
def test_emulated_combine_bs_pass_major(L, G, P, offs, lean, pf2, xcd, jump):
    """Every payload pass in one launch (qf_combine_bs_r16_pm): workgroup
    range p runs pass p with its records at coef + p * pass_stride and its
    outputs at rows 16 p ..; generations with fewer outputs leave the later
    passes' rows untouched. xcd: the interleaved form (qf_combine_bs_r16_pmx),
    pass (w >> 3) mod P of workgroup w, on a grid of 8 slots per pass; jump:
    the products as calls into the coefficient blocks (KernelSpec.cmb_jump)."""
    global _GFT
    if _GFT is None:
        _GFT = _gf_table()
    rng = np.random.default_rng(L + G + P)
    spec = bs.KernelSpec(0, 16, mode="cmb", pass_major=True, cmb_lean=lean, cmb_pf2=pf2, pm_xcd=xcd, cmb_jump=jump)
    Lp = (L + 15) // 16 * 16
    rs, drs = Lp + 32, Lp + 48
    nslot = 16 * P + 4
    rgs, dgs = nslot * rs + 16, 16 * P * drs + 32
    cgs = (nslot + 1) * 16
    PS = G * cgs + 64                       # the records' pass stride
    rows = rng.integers(0, 256, G * rgs, dtype=np.uint8)
    rec = rng.integers(0, 256, P * PS, dtype=np.uint8)
    e = rng.integers(1, 16 * P + 1, G).astype(np.uint32)
    bound = rng.integers(1, nslot + 1, G).astype(np.uint32)
    e[0] = 16 * P
    out = np.full(G * dgs, 0xEE, np.uint8)
    ROWS, OUT, REC, NO, BD, TAB, T1, T2 = (0x10000000, 0x40000000, 0x50000000, 0x60000000, 0x61000000,
                                           0x62000000, 0x63000000, 0x64000000)
    emu = bs.Emulator(bs.generate(spec))
    so = do = 0
    rgs_k, dgs_k = rgs, dgs
    if offs:
        emu.add_buffer(T1, np.array([(G - 1 - g) * rgs for g in range(G)], np.uint64).view(np.uint8))
        emu.add_buffer(T2, np.array([(G - 1 - g) * dgs for g in range(G)], np.uint64).view(np.uint8))
        so, do, rgs_k, dgs_k = T1, T2, 0, 0
    for base, buf in ((ROWS, rows), (OUT, out), (REC, rec), (NO, e), (BD, bound),
                      (TAB, bs.cmb_index_table().reshape(-1).view(np.uint8))):
        emu.add_buffer(base, buf.view(np.uint8))
    n = 8 if xcd else 2                     # workgroups per pass (persistent: items stride 4 n waves)
    ka, n_items = bs.cmb_kernargs(ROWS, OUT, rgs_k, dgs_k, rs, drs, REC, cgs, 0, NO, BD, TAB, L, G, 4 * n,
                                  rows_offs=so, dst_offs=do, pass_stride=PS, pm_xcd_passes=P if xcd else 0)
    for wg in range(P * n):
        for w in range(4):
            emu.run_wave(ka, wg, w)
    for g in range(G):
        gr = (G - 1 - g) if offs else g
        blk = out[gr * dgs:(gr + 1) * dgs]
        for j in range(16 * P):
            row = blk[j * drs:(j + 1) * drs]
            if j < e[g]:
                p, jj = divmod(j, 16)
                want = np.zeros(L, np.uint8)
                for sl in range(int(bound[g])):
                    c = rec[p * PS + g * cgs + 16 * sl + jj]
                    want ^= _GFT[c][rows[gr * rgs + sl * rs: gr * rgs + sl * rs + L]]
                assert (row[:L] == want).all(), (g, j)
                assert (row[L:] == 0xEE).all(), (g, j)
            else:
                assert (row == 0xEE).all(), (g, j)


@pytest.mark.parametrize("lean,jump", [(False, 0), (True, 0), (True, 3), (True, 2)])
@pytest.mark.parametrize("L,G,offs", [(1200, 6, False), (4100, 3, True), (100, 9, False), (33, 4, True)])
def test_emulated_combine_bs_wide(L, G, offs, lean, jump):
    """The wide single pass (qf_combine_bs_r24, QF_COMBINE_WIDE): 24 outputs
    per item, outputs 16..23 from the row's pass-1 record at coef +
    pass_stride; byte-equal to the two 16-output passes it replaces, and rows
    past a generation's e untouched."""
    global _GFT
    if _GFT is None:
        _GFT = _gf_table()
    rng = np.random.default_rng(L + 7 * G)
    spec = bs.KernelSpec(0, bs.CMB_WIDE_R, mode="cmb", cmb_lean=lean, cmb_jump=jump)
    assert spec.next_free_vgpr <= 256
    Lp = (L + 15) // 16 * 16
    rs, drs = Lp + 32, Lp + 48
    nslot = 28
    rgs, dgs = nslot * rs + 16, 24 * drs + 32
    cgs = (nslot + 1) * 16
    PS = G * cgs + 64
    rows = rng.integers(0, 256, G * rgs, dtype=np.uint8)
    rec = rng.integers(0, 256, 2 * PS, dtype=np.uint8)
    e = rng.integers(1, 25, G).astype(np.uint32)
    bound = rng.integers(1, nslot + 1, G).astype(np.uint32)
    e[0], e[1 % G] = 24, 17
    if G > 3:
        e[2], bound[3] = 16, 0
    out = np.full(G * dgs, 0xEE, np.uint8)
    ROWS, OUT, REC, NO, BD, TAB, T1, T2 = (0x10000000, 0x40000000, 0x50000000, 0x60000000, 0x61000000,
                                           0x62000000, 0x63000000, 0x64000000)
    emu = bs.Emulator(bs.generate(spec))
    so = do = 0
    rgs_k, dgs_k = rgs, dgs
    if offs:
        emu.add_buffer(T1, np.array([(G - 1 - g) * rgs for g in range(G)], np.uint64).view(np.uint8))
        emu.add_buffer(T2, np.array([(G - 1 - g) * dgs for g in range(G)], np.uint64).view(np.uint8))
        so, do, rgs_k, dgs_k = T1, T2, 0, 0
    for base, buf in ((ROWS, rows), (OUT, out), (REC, rec), (NO, e), (BD, bound),
                      (TAB, bs.cmb_index_table().reshape(-1).view(np.uint8))):
        emu.add_buffer(base, buf.view(np.uint8))
    n = 2
    ka, n_items = bs.cmb_kernargs(ROWS, OUT, rgs_k, dgs_k, rs, drs, REC, cgs, 0, NO, BD, TAB, L, G, 4 * n,
                                  rows_offs=so, dst_offs=do, pass_stride=PS)
    for wg in range(n):
        for w in range(4):
            emu.run_wave(ka, wg, w)
    for g in range(G):
        gr = (G - 1 - g) if offs else g
        blk = out[gr * dgs:(gr + 1) * dgs]
        for j in range(24):
            row = blk[j * drs:(j + 1) * drs]
            if j < e[g]:
                p, jj = divmod(j, 16)
                want = np.zeros(L, np.uint8)
                for sl in range(int(bound[g])):
                    c = rec[p * PS + g * cgs + 16 * sl + jj]
                    want ^= _GFT[c][rows[gr * rgs + sl * rs: gr * rgs + sl * rs + L]]
                assert (row[:L] == want).all(), (g, j)
                assert (row[L:] == 0xEE).all(), (g, j)
            else:
                assert (row == 0xEE).all(), (g, j)


# --------------------------------------------------------------------------
# Additive-FFT row loop (lch_fft.py, KernelSpec.fft)
# --------------------------------------------------------------------------
@pytest.mark.parametrize("k,r,ch", [(64, 16, 8), (64, 10, 8), (32, 16, 8), (16, 16, 8), (64, 16, 4),
                                    (64, 16, 16), (32, 5, 8), (128, 16, 8), (16, 1, 8)])
def test_lch_plan_equals_cauchy(k, r, ch):
    """The chunked additive-FFT schedule gives the reference's repairs
    p_j = sum_i inv(i ^ (k + j)) x_i (decoder.rs:280-298) on random bytes,
    for the canonical basis and the searched ones."""
    from quicfuscate_amd import lch_fft

    rng = np.random.default_rng(k * r + ch)
    plans = [lch_fft.plan(k, r, ch, check=0)]
    if (k, r, ch) in lch_fft.BEST:
        plans.append(lch_fft.best_plan(k, r, ch))
    C = bs.cauchy(k, r)
    for p in plans:
        for _ in range(6):
            x = rng.integers(0, 256, k).tolist()
            want = [0] * r
            for j in range(r):
                for i in range(k):
                    want[j] ^= bs.gf_mul(C[j][i], x[i])
            assert p.evaluate(x) == want


def test_lch_plan_is_cheaper_than_blocks():
    """The bench shape's plan costs fewer plane ops than one coefficient
    block per repair (8 r v_bitop3 + 22 combinations per row)."""
    from quicfuscate_amd import lch_fft

    p = lch_fft.best_plan(64, 16, 8)
    assert p.cost() + 64 * 48 < 64 * (48 + 22 + 8 * 16) * 0.7


@pytest.mark.parametrize("k,r,pd,L,G,zero_tail,defer", [
    (64, 16, 3, 1200, 2, True, 0),     # the benchmark kernel (zero tail, units of two generations)
    (64, 16, 3, 96, 5, False, 0),      # several generations per wave
    (64, 10, 3, 80, 3, True, 2),       # half chunks, r < R, deferred chunk folds
    (32, 16, 2, 1201, 2, True, 3),     # partial last unit
    (16, 16, 4, 64, 6, False, 1),
])
def test_emulated_fft_encode(oracle, k, r, pd, L, G, zero_tail, defer):
    spec = bs.KernelSpec(k, r, pd, fft=8, fft_defer=defer)
    ops = bs.generate(spec)
    Lv = bs.padded_units(L) if zero_tail else None
    rng = np.random.default_rng(k + 7 * L + G)
    srs = L + 16 * (k % 2)
    sgs = k * srs + 16
    drs = 16 * (Lv or L // 16) + 128
    dgs = r * drs
    src = rng.integers(0, 256, G * sgs, dtype=np.uint8)
    dst = np.full(G * dgs, 0xEE, np.uint8)
    emu = bs.Emulator(ops)
    emu.add_buffer(0x10000000, src)
    emu.add_buffer(0x40000000, dst)
    _, _, items = bs.launch_geometry(L, G, Lv)
    waves = (items + 3) // 4
    ka = bs.kernargs(0x10000000, 0x40000000, sgs, dgs, srs, drs, L, G, waves * 4, Lv=Lv, zero_tail=zero_tail)
    for wg in range(waves):
        for w in range(4):
            emu.run_wave(ka, wg, w)
    for g in range(G):
        rows = np.stack([src[g * sgs + i * srs: g * sgs + i * srs + L] for i in range(k)])
        want = oracle.encode(rows, r)
        for j in range(r):
            off = g * dgs + j * drs
            assert (dst[off: off + L] == want[j]).all(), (g, j)
            tail = 16 * Lv if zero_tail else L
            assert (dst[off + L: off + tail] == 0).all()
            assert (dst[off + tail: off + drs] == 0xEE).all()


@pytest.mark.parametrize("k,r,L,G,seed,erase,offs,es,lds", [
    (64, 16, 1200, 3, 1, 13, False, True, 0),   # the C3 shape, library options
    (64, 16, 1200, 2, 8, 13, False, False, 9),  # rows staged in LDS (global_load_lds), compact tables
    (64, 16, 96, 6, 2, None, True, True, 0),    # random e, offset tables
    (64, 16, 80, 5, 3, 16, False, True, 6),     # e = r: every block a pivot
    (64, 16, 1201, 2, 4, 5, False, True, 0),    # partial last unit
    (64, 10, 320, 4, 5, None, False, False, 0),  # r < R
    (16, 16, 96, 4, 6, 16, False, True, 0),
    (32, 16, 64, 5, 7, 0, False, True, 0),      # nothing erased
    # hybrid plans (k not a power of two: sources past 2^a in extra chunks / direct rows)
    (96, 15, 1200, 2, 9, 12, False, True, 0),
    (96, 15, 9000, 1, 10, None, True, True, 0),  # C5 row length, partial last unit
    (48, 8, 1200, 3, 11, None, False, True, 0),
])
def test_emulated_fft_fused_decode(oracle, k, r, L, G, seed, erase, offs, es, lds):
    """The additive-FFT fused decode (syndromes through the chunked
    transform, LU in registers): early stores (each recovered row as soon as
    back-substitution finishes it) and LDS-staged rows included.  The
    early-store cases run the library's kernel options since round 4
    (interleaved LU products, 64-bit-shift transposes and selectors)."""
    lib4 = {"lu_ilp": True, "bfi_transpose": "s64"} if es and not lds else {}
    assert _dec_case(oracle, k, r, 2, L, G, seed, erase, chunked=True, offs=offs, fft=8, early_stores=es,
                     lds_rows=lds, **lib4) == 0


@pytest.mark.parametrize("k,rt,R", [(128, 39, 16), (160, 48, 16), (196, 59, 16), (128, 20, 16), (24, 10, 16),
                                    (255, 1, 16), (17, 200, 16), (160, 48, 8), (100, 30, 8)])
def test_hybrid_plans_equal_cauchy(k, rt, R):
    """Every coset pass of a (k, r) code (lch_fft.coset_passes / hybrid_plan:
    sources [0, 2^a) through the FFT at the pass's coset, the rest direct)
    evaluates to the reference's repairs p_j = sum_i inv(i ^ (k + j)) x_i
    (decoder.rs:280-298) on random bytes; the passes tile 0 .. r - 1."""
    import random

    from quicfuscate_amd import lch_fft

    passes = lch_fft.coset_passes(k, rt, R)
    assert passes[0][0] == 0 and sum(n for _, n in passes) == rt
    assert all(j0 + n == j1 for (j0, n), (j1, _) in zip(passes, passes[1:]))
    rng = random.Random(k * 1000 + rt)
    for j0, n in passes:
        p = lch_fft.hybrid_plan(k, rt, j0, n, 8, R, check=0)
        for _ in range(3):
            xs = [rng.randrange(256) for _ in range(k)]
            want = [0] * n
            for j in range(n):
                for i in range(k):
                    want[j] ^= bs.gf_mul(bs.gf_inv(i ^ (k + j0 + j)), xs[i])
            assert p.evaluate(xs) == want, (j0, n)


@pytest.mark.parametrize("k,rt,L,G", [(24, 10, 200, 3), (20, 20, 72, 2), (48, 21, 64, 2), (160, 48, 40, 1),
                                     (40, 8, 100, 2), (96, 15, 40, 1)])
def test_emulated_fft_encode_hybrid_passes(oracle, k, rt, L, G):
    """Codes the plain additive-FFT plan does not cover (k not a power of
    two, repairs past the first coset): one kernel per coset pass
    (lch_fft.coset_passes), sources [0, 2^a) through the FFT at the pass's
    coset, the rest folded in directly; every pass writes its own repairs."""
    from quicfuscate_amd import lch_fft

    Lv = bs.padded_units(L)
    rng = np.random.default_rng(k * 13 + rt + L)
    srs = (L + 15) // 16 * 16 + 16 * (k % 2)
    sgs = k * srs
    drs = 16 * Lv + 64
    dgs = rt * drs
    src = rng.integers(0, 256, G * sgs + 64, dtype=np.uint8)
    dst = np.full(G * dgs, 0xEE, np.uint8)
    SRC, DST = 0x10000000, 0x40000000
    _, _, items = bs.launch_geometry(L, G, Lv)
    waves = (items + 3) // 4
    for j0, rp in lch_fft.coset_passes(k, rt):
        spec = bs.KernelSpec(k, rp, 2, r_total=rt, j0=j0, fft=8)
        emu = bs.Emulator(bs.generate(spec))
        emu.add_buffer(SRC, src)
        emu.add_buffer(DST, dst)
        ka = bs.kernargs(SRC, DST + j0 * drs, sgs, dgs, srs, drs, L, G, waves * 4, Lv=Lv, zero_tail=True)
        for wg in range(waves):
            for w in range(4):
                emu.run_wave(ka, wg, w)
    for g in range(G):
        rows = np.stack([src[g * sgs + i * srs: g * sgs + i * srs + L] for i in range(k)])
        want = oracle.encode(rows, rt)
        for j in range(rt):
            off = g * dgs + j * drs
            assert (dst[off: off + L] == want[j]).all(), (g, j)
            assert (dst[off + L: off + 16 * Lv] == 0).all(), (g, j)
            assert (dst[off + 16 * Lv: off + drs] == 0xEE).all()


@pytest.mark.parametrize("early", [0, 5])
@pytest.mark.parametrize("k,rt,L,G,blocks,helpers", [(24, 10, 200, 3, 0, 0), (48, 21, 2100, 2, 3, 0),
                                                    (20, 20, 72, 2, 0, 0), (196, 59, 40, 1, 0, 0),
                                                    (160, 48, 40, 1, 0, 0), (128, 39, 100, 2, 1, 0),
                                                    (160, 48, 40, 1, 0, 1), (20, 20, 72, 2, 1, 2),
                                                    (128, 20, 40, 1, 0, 0)])
def test_emulated_merged_passes_xchg(oracle, k, rt, L, G, blocks, helpers, early):
    """The merged additive-FFT encode whose waves share the row work through
    LDS (merged_spec(xchg=True), _generate_enc_xchg): wave w produces groups
    w, w + W, ... into its LDS slot, every wave folds every group; the
    workgroup's waves run together (shared LDS, s_barrier), persistent grids
    included; every repair byte equals the oracle's."""
    from quicfuscate_amd import lch_fft

    Lv = bs.padded_units(L)
    rng = np.random.default_rng(k * 19 + rt + L)
    srs = (L + 15) // 16 * 16 + 16 * (k % 2)
    sgs = k * srs
    drs = 16 * Lv + 64
    dgs = rt * drs
    src = rng.integers(0, 256, G * sgs + 64, dtype=np.uint8)
    dst = np.full(G * dgs, 0xEE, np.uint8)
    passes = [bs.KernelSpec(k, rp, 3, r_total=rt, j0=j0, fft=8, ld_policy="", xchg_early=early)
              for j0, rp in lch_fft.coset_passes(k, rt)]
    ms = bs.merged_spec(passes, xchg=True, helpers=helpers)
    assert ms.waves == len(passes) + helpers and len(passes) > 1 and ms.lds_bytes == ms.waves * 8 * bs.LDS_ROW_BYTES
    emu = bs.Emulator(bs.generate(ms))
    SRC, DST = 0x10000000, 0x40000000
    emu.add_buffer(SRC, src)
    emu.add_buffer(DST, dst)
    _, _, items = bs.launch_geometry(L, G, Lv)
    wgs = blocks or items
    ka = bs.kernargs(SRC, DST, sgs, dgs, srs, drs, L, G, wgs, Lv=Lv, zero_tail=True)
    for wg in range(wgs):
        emu.run_workgroup(ka, wg, ms.waves, ms.lds_bytes)
    for g in range(G):
        rows = np.stack([src[g * sgs + i * srs: g * sgs + i * srs + L] for i in range(k)])
        want = oracle.encode(rows, rt)
        for j in range(rt):
            off = g * dgs + j * drs
            assert (dst[off: off + L] == want[j]).all(), (g, j)
            assert (dst[off + L: off + 16 * Lv] == 0).all(), (g, j)
            assert (dst[off + 16 * Lv: off + drs] == 0xEE).all()


@pytest.mark.parametrize("k,rt,L,G,fft,blocks,lds", [(24, 10, 200, 3, 8, 0, 0), (20, 20, 72, 2, 0, 0, 0),
                                                      (48, 21, 4000, 2, 8, 3, 0), (40, 30, 40, 1, 0, 0, 0),
                                                      (160, 48, 40, 1, 8, 0, 0), (48, 21, 2100, 2, 8, 0, 6),
                                                      (196, 59, 40, 1, 8, 0, 0)])
def test_emulated_merged_passes(oracle, k, rt, L, G, fft, blocks, lds):
    """All passes of a code in one dispatch (MergedSpec): wave p of each
    workgroup runs pass p on the workgroup's item; a persistent grid (fewer
    workgroups than items, item stride = workgroups) included."""
    from quicfuscate_amd import lch_fft

    Lv = bs.padded_units(L)
    rng = np.random.default_rng(k * 17 + rt + L)
    srs = (L + 15) // 16 * 16 + 16 * (k % 2)
    sgs = k * srs
    drs = 16 * Lv + 64
    dgs = rt * drs
    src = rng.integers(0, 256, G * sgs + 64, dtype=np.uint8)
    dst = np.full(G * dgs, 0xEE, np.uint8)
    if fft:
        passes = [bs.KernelSpec(k, rp, 2, r_total=rt, j0=j0, fft=fft, lds_rows=lds)
                  for j0, rp in lch_fft.coset_passes(k, rt)]
    else:
        n = -(-rt // 12)
        cuts = [rt * p // n for p in range(n + 1)]
        passes = [bs.KernelSpec(k, cuts[p + 1] - cuts[p], 2, r_total=rt, j0=cuts[p]) for p in range(n)]
    ms = bs.merged_spec(passes)
    assert ms.waves == len(passes) > 1
    emu = bs.Emulator(bs.generate(ms))
    SRC, DST = 0x10000000, 0x40000000
    emu.add_buffer(SRC, src)
    emu.add_buffer(DST, dst)
    _, _, items = bs.launch_geometry(L, G, Lv)
    wgs = blocks or items
    ka = bs.kernargs(SRC, DST, sgs, dgs, srs, drs, L, G, wgs, Lv=Lv, zero_tail=True)
    for wg in range(wgs):
        if lds:   # the waves of a workgroup share its LDS (row slots at s29)
            emu.run_workgroup(ka, wg, ms.waves, ms.lds_bytes)
        else:
            for w in range(ms.waves):
                emu.run_wave(ka, wg, w)
    for g in range(G):
        rows = np.stack([src[g * sgs + i * srs: g * sgs + i * srs + L] for i in range(k)])
        want = oracle.encode(rows, rt)
        for j in range(rt):
            off = g * dgs + j * drs
            assert (dst[off: off + L] == want[j]).all(), (g, j)
            assert (dst[off + L: off + 16 * Lv] == 0).all(), (g, j)
            assert (dst[off + 16 * Lv: off + drs] == 0xEE).all()


def test_emulated_fft_fused_decode_tab32(oracle):
    """Lab option lab_tab32: the split tables at a 32-B record stride in LDS
    (the table copy and the LU's address scaling follow spec.tab_stride)."""
    assert _dec_case(oracle, 64, 16, 2, 1200, 2, 21, 13, chunked=True, fft=8, early_stores=True, lu_ilp=True,
                     bfi_transpose="s64", lab_tab32=True) == 0


@pytest.mark.parametrize("k,r,L,G,seed,erase", [(32, 5, 1200, 3, 12, None), (32, 5, 9000, 1, 13, 5), (16, 4, 96, 4, 14, 3)])
def test_emulated_fft_fused_decode_chunk4(oracle, k, r, L, G, seed, erase):
    """The additive-FFT fused decode with chunks of 4 rows (fft=4: a ring of 6
    rows, 160 VGPRs at (32, 5), so three waves per SIMD; the LU's r column
    quads must fit that ring, r <= 8)."""
    assert _dec_case(oracle, k, r, 2, L, G, seed, erase, chunked=True, fft=4, early_stores=True, lu_ilp=True,
                     bfi_transpose="s64") == 0


@pytest.mark.parametrize("k,r,L,G,seed,erase", [(64, 16, 1200, 3, 11, 13), (64, 16, 80, 5, 12, 16),
                                                (64, 10, 320, 4, 13, None), (32, 16, 64, 5, 14, 0)])
def test_emulated_fft_fused_decode_lu_ahead(oracle, k, r, L, G, seed, erase):
    """Split-table reads two coefficients ahead of the LU products (three
    table buffers, lu_ahead = 2) on the library's options."""
    assert _dec_case(oracle, k, r, 2, L, G, seed, erase, chunked=True, fft=8, early_stores=True, lu_ilp=True,
                     bfi_transpose="s64", lu_ahead=2) == 0


def test_library_kernels_register_budget():
    """Every generated kernel the library embeds (build_lib.kernel_specs):
    each VGPR it names lies below its descriptor's next_free_vgpr, and every
    register tuple starts at an even register (gfx950)."""
    import re

    from quicfuscate_amd.build_lib import kernel_specs

    for spec in kernel_specs():
        if spec.mode == "cmb":
            continue
        text = bs.emit_asm(spec, bs.generate(spec)).split(".amdhsa_kernel", 1)[0]
        hi = 0
        for m in re.finditer(r"\bv(\d+)\b|v\[(\d+):(\d+)\]", text):
            if m.group(1):
                hi = max(hi, int(m.group(1)))
            else:
                lo, top = int(m.group(2)), int(m.group(3))
                assert lo % 2 == 0, (spec.name, m.group(0))
                hi = max(hi, top)
        assert hi < spec.next_free_vgpr <= 256, (spec.name, hi, spec.next_free_vgpr)


@pytest.mark.parametrize("k,r,mode", [(64, 16, "enc"), (64, 16, "dec"), (32, 16, "dec"), (16, 16, "enc")])
def test_fft_register_budget_covers_code(k, r, mode):
    """Every VGPR the FFT kernels name lies below the descriptor's
    next_free_vgpr (<= 256: two waves per SIMD), and register tuples are even."""
    import re

    spec = bs.KernelSpec(k, r, 2 if mode == "dec" else 3, mode, chunked=mode == "dec", fft=8)
    text = bs.emit_asm(spec, bs.generate(spec))
    hi = 0
    for m in re.finditer(r"\bv(\d+)\b|v\[(\d+):(\d+)\]", text):
        if m.group(1):
            hi = max(hi, int(m.group(1)))
        else:
            lo, top = int(m.group(2)), int(m.group(3))
            assert lo % 2 == 0, m.group(0)
            hi = max(hi, top)
    assert hi < spec.next_free_vgpr <= 256


def test_dec_lab_variants_stay_in_bounds():
    """tools/dec_lab.py's round-5 access-pattern variants (nodata, slot order,
    masked absent rows) are timing-only kernels, but they run on the GPU box:
    every load and store must stay inside the lab's buffers (the emulator
    raises on any access outside them).  C3 geometry, a few generations."""
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "tools"))
    import dec_lab
    from bs_lab import variant_ops

    k, r, L, e, G = 64, 16, 1200, 13, 6
    n_slots = k - e + r
    erased, smap = dec_lab.c3_inputs(G, k, r, L, e)
    recs = np.stack([bs.lu_record(k, r, list(range(e)), erased[g].tolist()) for g in range(G)])
    rows = np.random.default_rng(1).integers(0, 256, G * n_slots * L, dtype=np.uint8)
    ROWS, OUT, MAP, ZERO, REC, TAB = 0x10000000, 0x40000000, 0x70000000, 0x78000000, 0x7C000000, 0x7E000000
    Q = ((L + 15) // 16 + 1) // 2
    STAMPS = 0x7F000000
    outs = {}
    cxrecs = np.stack([bs.cx_record(k, r, list(range(e)), erased[g].tolist()) for g in range(G)])
    for name, kw, flags in (dec_lab.VARIANTS_STAMPS + [("lib_ref", dict(dec_lab.LIB_DEC4), ())] + dec_lab.VARIANTS_CX
                            + dec_lab.VARIANTS + dec_lab.VARIANTS_R05AL + dec_lab.VARIANTS_R05Y + dec_lab.VARIANTS_R05G + dec_lab.VARIANTS_R05F + dec_lab.VARIANTS_R05E + dec_lab.VARIANTS_R05D + dec_lab.VARIANTS_R05C + dec_lab.VARIANTS_R05B
                             + dec_lab.VARIANTS_R05A):
        if name.endswith("_2") or name.endswith("_warm") or kw.get("rs"):
            continue
        kw2 = {a: b for a, b in kw.items() if a not in ("pd", "cap", "rs", "rrs", "Q")}
        spec = bs.KernelSpec(k, r, kw.get("pd", 3), "dec", **kw2)
        emu = bs.Emulator(variant_ops(bs, spec, set(flags)))
        rrs, Qv = kw.get("rrs", L), kw.get("Q")
        waves = ((G * (Qv or Q) + 63) // 64 + 3) // 4
        out = np.zeros(G * e * rrs, np.uint8)
        cx = kw.get("cx", False)
        for base, buf in ((ROWS, rows), (OUT, out), (MAP, smap.reshape(-1)), (ZERO, np.zeros(1216, np.uint8)),
                          (REC, (cxrecs if cx else recs).reshape(-1)), (TAB, bs.split_tables())):
            emu.add_buffer(base, buf)
        ka = bs.kernargs(ROWS, OUT, n_slots * L, e * rrs, L, rrs, L, G, waves * 4, smap=MAP,
                         map_stride=smap.shape[1], zero=ZERO, lu=(REC, bs.CX_REC_BYTES if cx else bs.LU_REC_BYTES),
                         tables=TAB, chunked=True, Q=Qv)
        if kw.get("lab_stamps"):   # the stamp buffer pointer follows the 128 kernarg bytes
            emu.add_buffer(STAMPS, np.zeros(128 * 4 * waves, np.uint8))
            ka += np.array([STAMPS, 0, 0, 0], np.uint32).tobytes()
            assert spec.offs_kernarg == bs.KERNARG_BYTES_DEC - 16 and len(ka) == spec.kernarg_bytes
        for wg in range(waves):
            for w in range(4):
                emu.run_wave(ka, wg, w)
        outs[name] = out
    # the stamps change nothing the kernel computes, nor does the closed-form solve
    assert (outs["st_lib"] == outs["lib_ref"]).all() and outs["lib_ref"].any()
    assert all((outs[n] == outs["lib_ref"]).all() for n in ("c_cx", "c_cx_l9", "c_cx_l10", "c_cx_l9_st"))


def test_xchg_streams_meet_at_every_barrier():
    """Every library kernel whose waves share row work through LDS (xchg,
    helper waves included): each wave's stream, from its pass label to the
    item loop's back-edge, holds the same number of s_barrier ops with no
    branch that could skip one (a skipped barrier would leave the other waves
    of the workgroup waiting on the GPU)."""
    from quicfuscate_amd import build_lib

    specs = [s for s in build_lib.kernel_specs() if isinstance(s, bs.MergedSpec) and s.passes[0].xchg]
    assert len(specs) >= 6
    for ms in specs:
        ops = bs.generate(ms)
        labels = {op.args[0]: n for n, op in enumerate(ops) if op.name == "label"}
        counts = []
        for p in range(ms.waves):
            start = labels[f".Lpass{p}"]
            end = labels.get(f".Lpass{p + 1}", len(ops))
            body = ops[start:end]
            counts.append(sum(op.name == "s_barrier" for op in body))
            # barriers sit outside every conditional region: the only forward
            # branches between the first and last barrier are the fold skips
            # (synw), whose targets lie before the next barrier
            bars = [n for n, op in enumerate(body) if op.name == "s_barrier"]
            blabels = {op.args[0]: n for n, op in enumerate(body) if op.name == "label"}
            for n in range(bars[0], bars[-1]):
                op = body[n]
                tgt = next((a for a in op.args if isinstance(a, str) and a.startswith(".L")), None)
                if tgt is None or op.name == "label":
                    continue
                t = blabels[tgt]
                assert t > n and not any(n < b < t for b in bars), (ms.name, p, op.name, tgt)
        assert len(set(counts)) == 1 and counts[0] > 0, (ms.name, counts)


def test_pm_xcd_word_divides_exactly():
    """The interleaved pass-major payload kernel's h div P = (h * magic) >> 16
    (kernarg word 33, bs_codegen.pm_xcd_word; qf_bs.hip computes the same
    word) is exact over every workgroup index the launch can produce."""
    for P in (2, 3, 4):
        w = bs.pm_xcd_word(P)
        assert w & 7 == P
        M = w >> 3
        assert all((h * M) >> 16 == h // P and h * M < 1 << 32 for h in range(1 << 15))


@pytest.mark.parametrize("L,G,P16,offs", [(1200, 5, 3, False), (4100, 3, 4, True), (100, 9, 4, False),
                                          (33, 6, 3, False), (2000, 7, 2, False)])
def test_emulated_combine_bs_pm24(L, G, P16, offs):
    """The 24-output pass-major payload pass with jump-table products
    (qf_combine_bs_r24_pm_j3): pass p' takes outputs 24 p' .. 24 p' + 23 from
    the 16-output record passes' bytes (three 8-byte pieces, a piece in an
    unwritten record pass redirected: its outputs lie past e_max); every
    generation's e outputs equal the 16-output passes' products, rows past e
    untouched."""
    global _GFT
    if _GFT is None:
        _GFT = _gf_table()
    rng = np.random.default_rng(L + 3 * G + P16)
    spec = bs.KernelSpec(0, bs.CMB_WIDE_R, mode="cmb", pass_major=True, cmb_lean=True, cmb_jump=3)
    assert spec.next_free_vgpr <= 256
    e_max = 16 * P16
    P24 = -(-e_max // 24)
    Lp = (L + 15) // 16 * 16
    rs, drs = Lp + 32, Lp + 48
    nslot = e_max + 4
    rgs, dgs = nslot * rs + 16, 24 * P24 * drs + 32
    cgs = (nslot + 1) * 16
    PS = G * cgs + 64
    rows = rng.integers(0, 256, G * rgs, dtype=np.uint8)
    rec = rng.integers(0, 256, P16 * PS, dtype=np.uint8)      # exactly the record passes written
    e = rng.integers(0, e_max + 1, G).astype(np.uint32)
    bound = rng.integers(1, nslot + 1, G).astype(np.uint32)
    e[0] = e_max
    if G > 2:
        e[1], e[2] = 24, 25
    out = np.full(G * dgs, 0xEE, np.uint8)
    ROWS, OUT, REC, NO, BD, TAB, T1, T2 = (0x10000000, 0x40000000, 0x50000000, 0x60000000, 0x61000000,
                                           0x62000000, 0x63000000, 0x64000000)
    emu = bs.Emulator(bs.generate(spec))
    so = do = 0
    rgs_k, dgs_k = rgs, dgs
    if offs:
        emu.add_buffer(T1, np.array([(G - 1 - g) * rgs for g in range(G)], np.uint64).view(np.uint8))
        emu.add_buffer(T2, np.array([(G - 1 - g) * dgs for g in range(G)], np.uint64).view(np.uint8))
        so, do, rgs_k, dgs_k = T1, T2, 0, 0
    for base, buf in ((ROWS, rows), (OUT, out), (REC, rec), (NO, e), (BD, bound),
                      (TAB, bs.cmb_index_table().reshape(-1).view(np.uint8))):
        emu.add_buffer(base, buf.view(np.uint8))
    n = 2
    ka, _ = bs.cmb_kernargs(ROWS, OUT, rgs_k, dgs_k, rs, drs, REC, cgs, 0, NO, BD, TAB, L, G, 4 * n,
                            rows_offs=so, dst_offs=do, pass_stride=PS)
    ka = ka[:-4] + np.uint32(P16).tobytes()                 # word 33: the record passes written
    for wg in range(P24 * n):
        for w in range(4):
            emu.run_wave(ka, wg, w)
    for g in range(G):
        gr = (G - 1 - g) if offs else g
        blk = out[gr * dgs:(gr + 1) * dgs]
        for j in range(24 * P24):
            row = blk[j * drs:(j + 1) * drs]
            if j < e[g]:
                p, jj = divmod(j, 16)
                want = np.zeros(L, np.uint8)
                for sl in range(int(bound[g])):
                    c = rec[p * PS + g * cgs + 16 * sl + jj]
                    want ^= _GFT[c][rows[gr * rgs + sl * rs: gr * rgs + sl * rs + L]]
                assert (row[:L] == want).all(), (g, j)
                assert (row[L:] == 0xEE).all(), (g, j)
            else:
                assert (row == 0xEE).all(), (g, j)


@pytest.mark.parametrize("L,G,zero_tail", [(320, 7, True), (1201, 4, True), (96, 9, False)])
def test_emulated_sliding_window_encoders(oracle, L, G, zero_tail):
    """The library's sliding-window encoders ('g', build_lib BS_SLIDING_*:
    cached row loads, (48, 8) as the hybrid FFT pass) on overlapping windows,
    generation stride = row stride (window g = rows g .. g + k - 1), every
    window's repairs equal the oracle's encode of its rows."""
    from quicfuscate_amd.build_lib import kernel_specs
    specs = [s for s in kernel_specs() if getattr(s, "sliding", False)]
    assert {(s.k, s.r) for s in specs} >= {(32, 5), (48, 8), (16, 1)}
    for spec in specs:
        k, r = spec.k, spec.r
        Lv = bs.padded_units(L) if zero_tail else None
        rng = np.random.default_rng(k + L + G)
        srs = (L + 15) // 16 * 16 + 16
        drs = 16 * (Lv or L // 16) + 128
        dgs = r * drs
        src = rng.integers(0, 256, (G + k - 1) * srs + 64, dtype=np.uint8)
        dst = np.full(G * dgs, 0xEE, np.uint8)
        emu = bs.Emulator(bs.generate(spec))
        emu.add_buffer(0x10000000, src)
        emu.add_buffer(0x40000000, dst)
        _, _, items = bs.launch_geometry(L, G, Lv)
        waves = (items + 3) // 4
        ka = bs.kernargs(0x10000000, 0x40000000, srs, dgs, srs, drs, L, G, waves * 4, Lv=Lv, zero_tail=zero_tail)
        for wg in range(waves):
            for w in range(4):
                emu.run_wave(ka, wg, w)
        for g in range(G):
            rows = np.stack([src[(g + i) * srs: (g + i) * srs + L] for i in range(k)])
            want = oracle.encode(rows, r)
            for j in range(r):
                off = g * dgs + j * drs
                assert (dst[off: off + L] == want[j]).all(), (spec.name, g, j)
                tail = 16 * Lv if zero_tail else L
                assert (dst[off + L: off + tail] == 0).all(), spec.name
