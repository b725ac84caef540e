"""GF(2^8) additive-FFT schedules (quicfuscate_amd/lch_fft.py) on scalars: the
transposed schedule and the closed-form Cauchy inverse behind DESIGN 3.2's
round-5 costing of a decode solve."""
def test_transposed_fft_schedule_is_cauchy_transpose():
    """DESIGN 3.2 (round 5) costing: the (64, 16) encode schedule run
    backwards with each op transposed computes C^T t, at the same op count."""
    import random
    from quicfuscate_amd import lch_fft as F
    p = F.best_plan(64, 16)
    k, r = 64, 16
    rng = random.Random(5)
    for _ in range(10):
        t = [rng.randrange(256) for _ in range(r)]
        want = [0] * k
        for i in range(k):
            for j in range(r):
                want[i] ^= F.mul(F.inv(i ^ (k + j)), t[j])
        assert F.transposed_evaluate(p, t) == want


def test_closed_form_cauchy_inverse():
    import random
    from quicfuscate_amd import lch_fft as F
    k, r = 64, 16
    rng = random.Random(6)
    for _ in range(30):
        e = rng.randrange(1, 17)
        E = sorted(rng.sample(range(k), e))
        J = sorted(rng.sample(range(r), e))
        alpha, beta = F.cauchy_inverse_factors(k, J, E)
        for b in range(e):
            for c in range(e):
                acc = 0
                for a in range(e):
                    d = F.mul(F.mul(alpha[b], beta[a]), F.inv((k + J[a]) ^ E[b]))
                    acc ^= F.mul(d, F.inv((k + J[a]) ^ E[c]))
                assert acc == (b == c)
