"""The Wiedemann oracle (oracle/qf_oracle_wiedemann.c, decoder.rs:794-975)
against the Gauss-Jordan oracle (k <= 256) and against the original bytes
(k > 256), plus the reference's own test shape (src/fec/mod.rs:142-176,
adaptive.rs:694-728: k = 260, packets 0 and 5 lost, 4 repairs).  CPU only."""
from __future__ import annotations

import numpy as np
import pytest

from tests import oracle_py as oracle


def _case(rng, k, e, L, extra=0, dup=False):
    """k sources, e of them lost, e + extra repairs with random coefficient
    rows; arrival = surviving sources in order, then the repairs."""
    src = rng.integers(0, 256, (k, L), dtype=np.uint8)
    lost = np.sort(rng.choice(k, e, replace=False))
    r = e + extra
    coef = rng.integers(0, 256, (r, k), dtype=np.uint8)
    rep = oracle.encode(src, r, coef)
    keep = [i for i in range(k) if i not in set(lost.tolist())]
    idx = keep + [k + j for j in range(r)]
    if dup:
        idx = keep[:3] + idx
    rows = np.concatenate([src[[i for i in idx if i < k]], rep]) if idx else np.zeros((0, L), np.uint8)
    rc = np.zeros((len(idx), k), np.uint8)
    rc[len(idx) - r:] = coef
    return src, lost, np.array(idx, np.uint16), rows, rc


@pytest.mark.parametrize("k,e,L", [(16, 3, 40), (64, 13, 64), (200, 20, 24), (256, 1, 8)])
def test_wiedemann_equals_gauss_jordan(k, e, L):
    rng = np.random.default_rng(k * 7 + e)
    src, lost, idx, rows, rc = _case(rng, k, e, L, extra=2)
    s1, out1, m1 = oracle.decode(k, idx, rows, rc)
    s2, out2, m2, tries = oracle.wiedemann(k, idx, rows, rc)
    assert s1 == s2 == oracle.OK
    assert (out1 == out2).all() and (m1 == m2).all() and (out2 == src).all()
    assert tries >= 1


@pytest.mark.parametrize("k,e,L", [(257, 1, 16), (260, 2, 8), (300, 7, 33), (512, 16, 12), (1024, 3, 4)])
def test_wiedemann_large_k_recovers_sources(k, e, L):
    rng = np.random.default_rng(k + e)
    src, lost, idx, rows, rc = _case(rng, k, e, L, extra=1)
    s, out, mask, tries = oracle.wiedemann(k, idx, rows, rc)
    assert s == oracle.OK, s
    assert (out == src).all()
    assert mask.sum() == k - e and not mask[lost].any()


def test_reference_wiedemann_path_shape():
    """mod.rs:142-176: k = 260, n = 264, make_packet payload data[0] = i % 256
    in 600-byte pool blocks, packets 0 and 5 not added, all 4 repairs added:
    the first 260 accepted rows (258 sources + 2 repairs) must decode.  The
    reference's Encoder cannot make these repairs (its u8 Cauchy rows hit
    gf_inv(0) at k = 260: SURVEY F5), so the repair rows here carry explicit
    random coefficients, which Decoder::add_packet takes as they come."""
    k, n, L = 260, 264, 600
    src = np.zeros((k, L), np.uint8)
    src[:, 0] = np.arange(k) % 256
    rng = np.random.default_rng(260)
    coef = rng.integers(1, 256, (n - k, k), dtype=np.uint8)
    rep = oracle.encode(src, n - k, coef)
    idx = [i for i in range(1, k) if i != 5] + [k + j for j in range(n - k)]
    rows = np.concatenate([src[[i for i in idx if i < k]], rep])
    rc = np.zeros((len(idx), k), np.uint8)
    rc[-(n - k):] = coef
    s, out, mask, _ = oracle.wiedemann(k, idx, rows, rc)
    assert s == oracle.OK
    assert (out[:, 0] == np.arange(k) % 256).all() and (out == src).all()
    # the reference's own repairs for this shape panic (gf_inv(0))
    s2, _, _, _ = oracle.wiedemann(k, idx, rows, None)
    assert s2 == oracle.ERANGE


def test_wiedemann_singular_and_not_ready():
    rng = np.random.default_rng(5)
    k, e, L = 300, 3, 16
    src, lost, idx, rows, rc = _case(rng, k, e, L)
    rc2 = rc.copy()
    rc2[-1] = rc2[-2]          # two equal repair rows: rank k - 1
    rows2 = rows.copy()
    rows2[-1] = rows2[-2]
    s, _, _, tries = oracle.wiedemann(k, idx, rows2, rc2)
    assert s == oracle.ERANK
    s, _, _, _ = oracle.wiedemann(k, idx[:-1], rows[:-1], rc[:-1])
    assert s == oracle.ENOTREADY
    # a zero repair row (all coefficients 0) is singular too
    rc3 = rc.copy()
    rc3[-1] = 0
    s, _, _, _ = oracle.wiedemann(k, idx, rows, rc3)
    assert s == oracle.ERANK


def test_wiedemann_duplicates_and_no_loss():
    rng = np.random.default_rng(9)
    k, L = 270, 10
    src, lost, idx, rows, rc = _case(rng, k, 4, L, dup=True)
    s, out, _, _ = oracle.wiedemann(k, idx, rows, rc)
    assert s == oracle.OK and (out == src).all()
    src, lost, idx, rows, rc = _case(rng, k, 0, L)
    s, out, mask, _ = oracle.wiedemann(k, idx, rows, rc)
    assert s == oracle.OK and (out == src).all() and mask.all()


def _diag_case(k, L, seed, zero_at=None):
    """Every source lost, repair p = c_p * source p: A = diag(c).  c_p = 7 on
    rows {0, 1, 16, 17} and 11 elsewhere: the init vectors u_i = (i + b + 1)
    % 255 XOR to zero over {0, 1, 16, 17} for every b < 8, so no projection
    sees the eigenvalue 7 and every try fails verification (or is a zero
    sequence) although A is nonsingular."""
    rng = np.random.default_rng(seed)
    src = rng.integers(0, 256, (k, L), dtype=np.uint8)
    c = np.full(k, 11, np.uint8)
    c[[0, 1, 16, 17]] = 7
    if zero_at is not None:
        c[zero_at] = 0
    rc = np.zeros((k, k), np.uint8)
    rc[np.arange(k), np.arange(k)] = c
    rows = oracle.encode(src, k, rc)
    return src, [k + p for p in range(k)], rows, rc


def test_wiedemann_exact_fallback():
    """qf_oracle_wiedemann.c: when no init vector verifies, exact elimination
    decides -- a nonsingular system decodes (tries = 9), a singular one is
    ERANK.  (The reference returns its unchecked W here; parity with it is
    the decoded sources, which are unique.)"""
    for k in (20, 64):
        src, idx, rows, rc = _diag_case(k, 24, k)
        s, out, mask, tries = oracle.wiedemann(k, idx, rows, rc)
        assert s == oracle.OK and tries == 9
        assert (out == src).all() and not mask.any()
    src, idx, rows, rc = _diag_case(20, 24, 3, zero_at=5)
    s, _, _, _ = oracle.wiedemann(20, idx, rows, rc)
    assert s == oracle.ERANK
