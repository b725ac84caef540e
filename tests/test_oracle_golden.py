"""The CPU oracle pinned against the golden vectors and the reference's own
test contracts (CPU only).  SURVEY 8(c)."""
import hashlib
import json
from pathlib import Path

import numpy as np
import pytest

GOLDEN = json.loads((Path(__file__).parent / "golden" / "golden.json").read_text())


def pattern(k, L):
    i = np.arange(k)[:, None]
    t = np.arange(L)[None, :]
    return ((7 * i + 13 * t + 1) & 255).astype(np.uint8)


def test_tables_match_golden(oracle):
    e, lg = oracle.tables()
    assert e.tobytes().hex() == GOLDEN["exp"]
    assert lg.tobytes().hex() == GOLDEN["log"]
    assert list(e[:10]) == [1, 2, 4, 8, 16, 32, 64, 128, 29, 58]
    assert list(lg[1:9]) == [0, 1, 25, 2, 50, 26, 198, 3]


def test_kats(oracle):
    for a, b, p in GOLDEN["kat_mul"]:
        assert oracle.mul(a, b) == p
    for a, v in GOLDEN["kat_inv"]:
        assert oracle.inv(a) == v
    assert oracle.inv(0) is None  # gf_inv(0) panics in the reference


def test_mul_table_exhaustive_equals_shift_and_add(oracle):
    # mod.rs:177-187 / tests/fec.rs:262-272: gf_mul == gf_mul_table for all
    # 65,536 pairs; the shift-and-add multiply (gf_tables.rs:59-74) is an
    # independent restatement of the same field.
    t = oracle.mul_table_full()
    for a in range(256):
        for b in range(0, 256, 17):
            assert t[a, b] == oracle.mul_shift(a, b)
    # field axioms on the whole table
    assert (t == t.T).all()
    assert (t[1] == np.arange(256)).all()
    nz = t[1:, 1:]
    for row in nz:
        assert len(set(row.tolist())) == 255  # every nonzero element invertible


def test_clmul_fold_defect_documented(oracle):
    # the as-written CLMUL + fold agrees with the table on 718 pairs.
    agree = sum(1 for a in range(256) for b in range(256) if oracle.mul_clmul_fold(a, b) == oracle.mul(a, b))
    assert agree == GOLDEN["clmul_fold_agree_with_table"] == 718


@pytest.mark.parametrize("key", ["4x2", "10x2", "16x16", "64x16"])
def test_cauchy_golden(oracle, key):
    k, r = map(int, key.split("x"))
    assert oracle.cauchy(k, r).tobytes().hex() == GOLDEN["cauchy"][key]


def test_cauchy_sha_and_panics(oracle):
    for key, h in GOLDEN["cauchy_sha"].items():
        k, r = map(int, key.split("x"))
        assert hashlib.sha256(oracle.cauchy(k, r).tobytes()).hexdigest()[:32] == h
    for k, r, panics in GOLDEN["cauchy_panics"]:
        assert (oracle.cauchy(k, r) is None) == panics


def test_encode_golden(oracle):
    for name, v in GOLDEN["encode"].items():
        k, r, L = v["k"], v["r"], v["L"]
        src = pattern(k, L) if v["src"] == "pattern" else np.frombuffer(bytes.fromhex(v["src"]), np.uint8).reshape(k, L)
        rep = oracle.encode(src, r)
        if "rep" in v:
            assert rep.tobytes().hex() == v["rep"], name
        else:
            assert hashlib.sha256(rep.tobytes()).hexdigest()[:32] == v["rep_sha"], name


def test_encode_k4_known_answer(oracle):
    src = np.repeat(np.arange(4, dtype=np.uint8)[:, None], 8, axis=1)
    rep = oracle.encode(src, 2)
    assert (rep[0] == 128).all() and (rep[1] == 160).all()


@pytest.mark.parametrize("name", sorted(GOLDEN["decode"]))
def test_decode_reference_cases(oracle, name):
    v = GOLDEN["decode"][name]
    k, L = v["k"], v["L"]
    rows = np.frombuffer(bytes.fromhex(v["rows"]), np.uint8).reshape(-1, L)
    st, out, mask = oracle.decode(k, v["row_index"], rows)
    assert st == 0
    assert out.tobytes().hex() == v["expected"]
    # reference assertion: out[i].data[0] == i
    assert list(out[:, 0]) == [i & 0xFF for i in range(k)]


def test_as_written_decoder_defect(oracle):
    # decoder.rs:692 + 475-478 as written returns 186 for packet 1.
    v = GOLDEN["decode"]["fec_rs_gf8_encode_decode"]
    rows = np.frombuffer(bytes.fromhex(v["rows"]), np.uint8).reshape(-1, 8)
    st, out = oracle.decode_as_written(4, v["row_index"], rows)
    assert st == 0 and out[1, 0] == v["as_written_packet1_byte0"] == 186


def test_decode_edge_cases(oracle):
    rng = np.random.default_rng(1)
    k, r, L = 8, 4, 24
    src = rng.integers(0, 256, (k, L), dtype=np.uint8)
    rep = oracle.encode(src, r)
    # not enough rows
    st, _, _ = oracle.decode(k, [0, 1, 2, 8], np.vstack([src[:3], rep[:1]]))
    assert st == oracle.ENOTREADY
    # duplicate systematic rows are ignored, then repairs fill in
    idx = [0, 0, 1, 2, 3, 4, 5, 8, 9]
    rows = np.vstack([src[0], src[0], src[1:6], rep[:2]])
    st, out, mask = oracle.decode(k, idx, rows)
    assert st == 0 and (out == src).all() and list(mask) == [1] * 6 + [0, 0]
    # duplicate repair rows make the first-k matrix singular (decoder.rs:679)
    idx = [0, 1, 2, 3, 4, 5, 8, 8, 9]
    rows = np.vstack([src[:6], rep[0], rep[0], rep[1]])
    st, _, _ = oracle.decode(k, idx, rows)
    assert st == oracle.ERANK
    # all repairs, no systematic rows
    st, out, _ = oracle.decode(4, [4, 5, 6, 7], oracle.encode(src[:4], 4))
    assert st == 0 and (out == src[:4]).all()


def test_splitmix_golden(oracle):
    assert oracle.fill_splitmix(32, 0x51464543).tobytes().hex() == GOLDEN["splitmix_seed_QFEC_first32"]
    a = oracle.fill_splitmix(100, 7)
    b = oracle.fill_splitmix(60, 7, 5)
    assert (a[40:100] == b).all()


@pytest.mark.parametrize("kind", ["table", "avx2", "gfni"])
@pytest.mark.parametrize("k,r,L,G,threads", [(64, 16, 1200, 5, 3), (7, 5, 33, 4, 2), (16, 1, 31, 3, 1),
                                             (5, 3, 64, 2, 1), (9, 4, 129, 2, 2)])
def test_cpu_comparison_encoders_match_oracle(oracle, kind, k, r, L, G, threads):
    if not oracle.has_cpu_kind(kind):
        pytest.skip(f"no {kind} on this host")
    rng = np.random.default_rng(k + L)
    src = rng.integers(0, 256, (G, k, L), dtype=np.uint8)
    got = oracle.cpu_encode(kind, src, r, threads)
    for g in range(G):
        assert (got[g] == oracle.encode(src[g], r)).all()


def test_cpu_clmul_as_written_is_the_defective_fold(oracle):
    """cpu_encode("clmul") restates the reference's per-byte PCLMULQDQ path
    (gf_tables.rs:129-141 inside decoder.rs:228-259) for timing; its output
    must equal the same loop over the restated fold (oracle_gf_mul_clmul_fold),
    and differ from the correct table encode."""
    if not oracle.has_cpu_kind("clmul"):
        pytest.skip("no PCLMULQDQ on this host")
    k, r, L = 16, 4, 37
    rng = np.random.default_rng(3)
    src = rng.integers(0, 256, (2, k, L), dtype=np.uint8)
    got = oracle.cpu_encode("clmul", src, r, 2)
    for g in range(2):
        assert (got[g] == oracle.encode_clmul_fold(src[g], r)).all()
    assert not (got[0] == oracle.encode(src[0], r)).all()
    # the same product through the per-byte dispatch model (optimize.rs:385-408)
    assert (oracle.cpu_encode("clmul_dispatch", src, r, 2) == got).all()
