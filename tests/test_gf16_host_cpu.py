"""GF(2^16) host helpers of the product library (qf_gf16_mul / qf_gf16_inv /
qf_cauchy16_coeffs, gf_tables.rs:331-380, decoder.rs:77-80) against the
oracle and golden16.json.  No device calls."""
import json
from pathlib import Path

import numpy as np

G = json.loads((Path(__file__).parent / "golden" / "golden16.json").read_text())


def test_gf16_mul_inv_match_oracle(qf, oracle):
    for a, b, p in G["mul"]:
        assert qf.gf16_mul(a, b) == p
    for a, i in G["inv"]:
        assert qf.gf16_inv(a) == i
    rng = np.random.default_rng(3)
    for a, b in rng.integers(0, 65536, (2000, 2)).tolist():
        assert qf.gf16_mul(a, b) == oracle.mul16(a, b)
    for a in rng.integers(1, 65536, 300).tolist():
        assert qf.gf16_inv(a) == oracle.inv16(a)


def test_gf16_inv_zero_raises(qf):
    import pytest

    with pytest.raises(qf.QfError):
        qf.gf16_inv(0)


def test_cauchy16_matches_oracle(qf, oracle):
    assert qf.cauchy16_coefficients(8, 4) == G["cauchy_k8_r4"]
    assert np.array_equal(np.array(qf.cauchy16_coefficients(64, 16), np.uint16), oracle.cauchy16(64, 16))
    assert qf.cauchy16_coefficients(1024, 8)[0][:8] == G["cauchy_k1024_r8_row0_head"]
