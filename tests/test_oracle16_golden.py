"""The GF(2^16) oracle (oracle/qf_oracle16.c) against golden16.json
(independent Python restatement, tests/golden/gen_golden16.py) and the
reference's own contract tests/fec.rs:52-82 (gf16_encode_decode)."""
import hashlib
import json
from pathlib import Path

import numpy as np

G = json.loads((Path(__file__).parent / "golden" / "golden16.json").read_text())


def _h(chunks):
    d = hashlib.sha256()
    for c in chunks:
        d.update(bytes(c))
    return d.hexdigest()[:32]


def test_mul_inv_known_answers(oracle):
    for a, b, p in G["mul"]:
        assert oracle.mul16(a, b) == p
    for a, i in G["inv"]:
        assert oracle.inv16(a) == i
        assert oracle.mul16(a, i) == 1
    assert oracle.inv16(0) is None  # the reference panics


def test_field_axioms_sampled(oracle):
    rng = np.random.default_rng(5)
    for a, b, c in rng.integers(0, 65536, (300, 3)).tolist():
        assert oracle.mul16(a, b) == oracle.mul16(b, a)
        assert oracle.mul16(a, b ^ c) == oracle.mul16(a, b) ^ oracle.mul16(a, c)
        assert oracle.mul16(oracle.mul16(a, b), c) == oracle.mul16(a, oracle.mul16(b, c))
    # 2 generates the multiplicative group (0x1100B is primitive)
    x, seen = 1, 0
    for i in range(1, 65536):
        x = oracle.mul16(x, 2)
        if x == 1:
            seen = i
            break
    assert seen == 65535


def test_cauchy16(oracle):
    assert oracle.cauchy16(8, 4).tolist() == G["cauchy_k8_r4"]
    c = oracle.cauchy16(64, 16)
    assert _h(int(v).to_bytes(2, "big") for v in c.reshape(-1)) == G["cauchy_k64_r16_sha"]
    assert oracle.cauchy16(1024, 8)[0, :8].tolist() == G["cauchy_k1024_r8_row0_head"]
    assert oracle.cauchy16(65535, 2) is None  # k + r > 65536: gf16_inv(0)


def test_encode16_known_answers(oracle):
    k, n, L = 8, 12, 8
    src = np.array([[i % 255] * L for i in range(k)], np.uint8)
    assert oracle.encode16(src, n - k).tolist() == G["fec_rs_gf16_repairs"]
    for k, r, L in ((16, 16, 1200), (64, 16, 1200)):
        src = np.array([[(7 * i + 13 * t + 1) & 255 for t in range(L)] for i in range(k)], np.uint8)
        assert _h(oracle.encode16(src, r)) == G[f"encode16_k{k}_r{r}_L{L}_sha"]


def test_reference_contract_gf16_encode_decode(oracle):
    """tests/fec.rs:52-82: k = 8, n = 12, packet 0 dropped, every source's
    first byte comes back."""
    k, n, L = 8, 12, 8
    src = np.array([[i % 255] * L for i in range(k)], np.uint8)
    rep = oracle.encode16(src, n - k)
    arrival = list(range(1, k)) + [k + j for j in range(n - k)]
    rows = np.stack([src[a] if a < k else rep[a - k] for a in arrival])
    st, out, mask = oracle.decode16(k, arrival, rows)
    assert st == 0
    assert out[:, 0].tolist() == G["fec_rs_gf16_decoded_first_bytes"] == [i % 255 for i in range(k)]
    assert (out == src).all()


def test_decode16_statuses(oracle):
    k, L = 6, 10
    rng = np.random.default_rng(9)
    src = rng.integers(0, 256, (k, L), dtype=np.uint8)
    rep = oracle.encode16(src, 4)
    # fewer than k rows
    assert oracle.decode16(k, [0, 1, 2], src[:3])[0] == -3
    # a duplicated systematic row is a row (Decoder16 does not filter): singular
    arr = [0, 0, 1, 2, 3, 4, 6]
    rows = np.stack([src[a] if a < k else rep[a - k] for a in arr])
    assert oracle.decode16(k, arr, rows)[0] == -4
    # random erasures decode to the sources
    for e in range(0, 5):
        er = sorted(rng.choice(k, e, replace=False).tolist())
        arr = [i for i in range(k) if i not in er] + [k + j for j in range(4)]
        rng.shuffle(arr)
        rows = np.stack([src[a] if a < k else rep[a - k] for a in arr])
        st, out, _ = oracle.decode16(k, arr, rows)
        if sum(a >= k for a in arr[:k]) == e:
            assert st == 0 and (out == src).all()
