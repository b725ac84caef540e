"""The CPU baseline rows of bench.py on the host (no GPU): the restated
gf_mul micro-loop of the reference's only published benchmark, and the
pinned C1 encoders against the oracle."""
import numpy as np
import pytest


@pytest.mark.parametrize("kind", ["table", "dispatch", "sse2", "avx512", "avx2"])
def test_gf_mul_micro_loop(oracle, kind):
    """benches/gf_bitslice_bench.rs:17-102: a[i] = i, b[i] = 255 - i over
    1,024 pairs; every product appears four times, so the XOR is 0 for the
    table product and for the reference's (defective) fold alike."""
    acc = oracle.gf_mul_loop(kind, 3)
    if acc == -3:
        pytest.skip(f"{kind} needs instructions this host lacks")
    assert acc == 0


@pytest.mark.parametrize("kind", ["avx512", "avx2"])
def test_clmul_members_agree_with_sse2(oracle, kind):
    """gf_mul_bitsliced_avx2 / _avx512 (gf_tables.rs:76-118) compute the same
    fold as gf_mul_bitsliced_sse2 (:129-141) on every operand pair."""
    if oracle.clmul_fold_pair(kind, 3, 7) == -3:
        pytest.skip(f"{kind} needs instructions this host lacks")
    for a in range(256):
        for b in range(0, 256, 5):
            assert oracle.clmul_fold_pair(kind, a, b) == oracle.clmul_fold_pair("sse2", a, b), (a, b)


def test_gf_mul_micro_loop_table_matches_products(oracle):
    # one pass of the table kind equals the XOR of the oracle's products
    want = 0
    for i in range(1024):
        want ^= oracle.mul(i & 0xFF, (255 - i) & 0xFF)
    assert oracle.gf_mul_loop("table", 1) == want


@pytest.mark.parametrize("r", [16, 1])
def test_c1_pinned_encoders_match_oracle(oracle, r):
    """BASELINE C1 shape (k = 16, L = 1200) on pinned worker threads."""
    rng = np.random.default_rng(r)
    src = rng.integers(0, 256, (9, 16, 1200), dtype=np.uint8)
    oracle.set_pinning(True)
    try:
        for kind in ("table", "gfni"):
            if not oracle.has_cpu_kind(kind):
                continue
            got = oracle.cpu_encode(kind, src, r, 4)
            for g in range(len(src)):
                assert (got[g] == oracle.encode(src[g], r)).all(), (kind, g)
    finally:
        oracle.set_pinning(False)
