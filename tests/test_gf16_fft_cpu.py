"""The additive-FFT GF(2^16) Cauchy encode (quicfuscate_amd/csrc/qf_gf16_fft.hip)
restated in numpy and checked against the oracle's Encoder16 (oracle/qf_oracle16.c,
decoder.rs:10-88 with the intended reduction) on the CPU.

For k = 2^a the sources sit on the subspace V = {0 .. k-1} of GF(2^16) and the
repair points k + j on its coset, so repair j = kappa * f(k + j) with f the
polynomial interpolating the sources over V (the GF(2^8) derivation of
quicfuscate_amd/lch_fft.py, same field-independent algebra).  The model uses
exactly the constants the library's host code derives from the table
W_q(2^m) (W_q = the subspace polynomial of {0 .. 2^q - 1}, GF(2)-linear):
    W_0(t) = t,  W_{q+1}(t) = W_q(t) (W_q(t) + W_q(2^q)),
    xhat(q, t) = W_q(t) / W_q(2^q),  Delta = prod_q W_q(2^q),  P_V(k) = W_a(k).
The device kernel runs the same butterflies in the log domain (Zech table;
tests/test_gpu_gf16.py), and the decode's solve reuses the transform
(test_fft_solve_recovers_erasures)."""
import numpy as np
import pytest

from quicfuscate_amd import gf16_codegen as g16

POLY = 0x1100B


def _tables():
    exp = np.zeros(2 * 65535, np.int64)
    log = np.full(65536, -1, np.int64)
    x = 1
    for i in range(65535):
        exp[i] = x
        log[x] = i
        x <<= 1
        if x & 0x10000:
            x ^= POLY
    exp[65535:] = exp[:65535]
    return exp, log


EXP, LOG = _tables()


def vmul(c: int, y: np.ndarray) -> np.ndarray:
    """c * y elementwise (y uint16 array)."""
    if c == 0:
        return np.zeros_like(y)
    out = EXP[(LOG[y.astype(np.int64)] + int(LOG[c])) % 65535].astype(np.uint16)
    out[y == 0] = 0
    return out


def smul(a: int, b: int) -> int:
    return g16.mul(a, b)


def constants(k: int, R: int):
    """(inv layers, fold * kappa, forward layers) as the host code computes them."""
    a, b = k.bit_length() - 1, R.bit_length() - 1
    W = [[1 << m for m in range(16)]]                       # W_0(2^m) = 2^m
    for q in range(a):
        wq = W[q][q]
        W.append([smul(w, w ^ wq) for w in W[q]])

    def w_at(q, t):
        v, m = 0, 0
        while t:
            if t & 1:
                v ^= W[q][m]
            t >>= 1
            m += 1
        return v

    def xhat(q, t):
        return smul(w_at(q, t), g16.inv(W[q][q]))

    inv_l = [[xhat(q, o) for o in range(0, k, 2 << q)] for q in range(a)]
    delta = 1
    for q in range(a):
        delta = smul(delta, W[q][q])
    kappa = smul(delta, g16.inv(w_at(a, k)))
    fk = []
    for i in range(k):
        f = kappa
        for q in range(b, a):
            if i >> q & 1:
                f = smul(f, xhat(q, k))
        fk.append(f)
    fwd_l = [[xhat(q, k ^ o) for o in range(0, R, 2 << q)] for q in range(b)]
    return inv_l, fk, fwd_l


def fft_encode(x: np.ndarray, k: int, r: int, first: int = 0) -> np.ndarray:
    """x: (k, n_sym) uint16 symbols -> repairs first .. first + r - 1, (r, n_sym)."""
    R = 1
    while R < first + r:
        R <<= 1
    a, b = k.bit_length() - 1, R.bit_length() - 1
    inv_l, fk, fwd_l = constants(k, R)
    y = x.astype(np.uint16).copy()
    for q in range(a):                                      # inverse transform over V
        h = 1 << q
        for blk, o in enumerate(range(0, k, 2 * h)):
            s = inv_l[q][blk]
            for i in range(o, o + h):
                y[i + h] ^= y[i]
                y[i] ^= vmul(s, y[i + h])
    d = np.zeros((R, x.shape[1]), np.uint16)
    for i in range(k):                                      # fold onto the coset, times kappa
        d[i % R] ^= vmul(fk[i], y[i])
    for q in reversed(range(b)):                            # forward transform over k + V_b
        h = 1 << q
        for blk, o in enumerate(range(0, R, 2 * h)):
            s = fwd_l[q][blk]
            for i in range(o, o + h):
                d[i] ^= vmul(s, d[i + h])
                d[i + h] ^= d[i]
    return d[first:first + r]


def to_sym(rows: np.ndarray) -> np.ndarray:
    return (rows[:, 0::2].astype(np.uint16) << 8) | rows[:, 1::2]


def to_bytes(sym: np.ndarray) -> np.ndarray:
    out = np.zeros((sym.shape[0], 2 * sym.shape[1]), np.uint8)
    out[:, 0::2] = sym >> 8
    out[:, 1::2] = sym & 0xFF
    return out


def test_recurrence_is_the_subspace_polynomial():
    # W_q(t) = prod_{u < 2^q} (t + u), checked directly for small q
    for q in range(4):
        for t in (1, 5, 0x1234, 0xFFFF):
            want = 1
            for u in range(1 << q):
                want = smul(want, t ^ u)
            W = [[1 << m for m in range(16)]]
            for qq in range(q):
                W.append([smul(w, w ^ W[qq][qq]) for w in W[qq]])
            got, m, tt = 0, 0, t
            while tt:
                if tt & 1:
                    got ^= W[q][m]
                tt >>= 1
                m += 1
            assert got == want, (q, t)


@pytest.mark.parametrize("k,r,first", [(2, 1, 0), (2, 2, 0), (4, 3, 0), (8, 8, 0), (16, 5, 0), (64, 16, 0),
                                       (64, 64, 0), (128, 96, 0), (256, 3, 100), (32, 7, 20), (512, 512, 0)])
def test_fft_matches_oracle(oracle, k, r, first):
    rng = np.random.default_rng(k * 31 + r + first)
    L = 6
    rows = rng.integers(0, 256, (k, L), dtype=np.uint8)
    rows[0, :2] = 0
    out = to_bytes(fft_encode(to_sym(rows), k, r, first))
    ref = oracle.encode16(rows, first + r)[first:]
    assert np.array_equal(out, ref)


@pytest.mark.parametrize("k,e", [(16, 5), (64, 33), (128, 128)])
def test_fft_solve_recovers_erasures(oracle, k, e):
    """The decode solve of qf_gf16_fft.hip (k_fft16_solve): with accepted
    repairs J (x_a = k + j_a) and erased sources E (y_b), the closed-form
    Cauchy inverse (C^-1)_ba = Qx_a Qy_b / ((x_a + y_b) Px_a Py_b) makes
        x_{E_b} = (Qy_b / Py_b) * FFT(z)[E_b],  z[j_a] = (Qx_a / Px_a) s_a,
    the same encode FFT with R = k (outputs on the whole coset).  Checked by
    recovering the erased sources from the oracle's repairs."""
    rng = np.random.default_rng(k * 7 + e)
    L = 4
    rows = rng.integers(0, 256, (k, L), dtype=np.uint8)
    x = to_sym(rows)
    E = sorted(rng.choice(k, e, replace=False).tolist())
    js = rng.choice(k, e, replace=False).tolist()          # accepted repairs k + j, j < k
    rep = to_sym(oracle.encode16(rows, k))                  # all k Cauchy rows
    known = np.ones(k, bool)
    known[E] = False
    xs = np.where(known[:, None], x, 0).astype(np.uint16)
    full = fft_encode(xs, k, k)                             # C[J, S] x_S for every repair
    s = [rep[j] ^ full[j] for j in js]                      # syndromes = C[J, E] x_E
    X = [k ^ j for j in js]

    def prod(vals):
        out = 1
        for v in vals:
            out = smul(out, v)
        return out

    z = np.zeros((k, x.shape[1]), np.uint16)
    for a, j in enumerate(js):
        qx = prod(X[a] ^ y for y in E)
        px = prod(X[a] ^ X[c] for c in range(e) if c != a)
        z[j] = vmul(smul(qx, g16.inv(px)), s[a])
    out = fft_encode(z, k, k)
    for b, y in enumerate(E):
        qy = prod(xa ^ y for xa in X)
        py = prod(y ^ E[c] for c in range(e) if c != b)
        assert np.array_equal(vmul(smul(qy, g16.inv(py)), out[y]), x[y]), (b, y)


# --- the bit-plane form of k_fft16_bs (qf_gf16_fft.hip) ---------------------
# A lane holds 32 symbol columns of a row as 16 plane dwords (plane p = bit p of
# every symbol).  Restated with numpy uint32 arrays: the load (byte swap of the
# two big-endian symbols of each dword + a 16 x 16 bit transpose of both dword
# halves), the product s x by Horner over the bits of s with x alpha = the
# planes shifted up and plane 15 folded into planes 0, 1, 3 and 12 (0x1100B),
# and the store (the transpose is its own inverse).

_M32 = np.uint32(0xFFFFFFFF)


def _bs_transpose(d: np.ndarray) -> np.ndarray:
    d = d.copy()
    for w, m in ((8, 0x00FF00FF), (4, 0x0F0F0F0F), (2, 0x33333333), (1, 0x55555555)):
        for i in range(16):
            if i & w:
                continue
            t = ((d[i] >> np.uint32(w)) ^ d[i + w]) & np.uint32(m)
            d[i + w] ^= t
            d[i] ^= (t << np.uint32(w)) & _M32
    return d


def _bs_swap16x2(w: np.ndarray) -> np.ndarray:
    return ((w & np.uint32(0x00FF00FF)) << np.uint32(8)) | ((w >> np.uint32(8)) & np.uint32(0x00FF00FF))


def _bs_load(row64: np.ndarray) -> np.ndarray:
    """64 bytes (32 big-endian symbols) -> 16 planes."""
    return _bs_transpose(_bs_swap16x2(row64.view("<u4").astype(np.uint32)))


def _bs_store(planes: np.ndarray) -> np.ndarray:
    return _bs_swap16x2(_bs_transpose(planes)).astype("<u4").view(np.uint8)


def _bs_mulx(x: np.ndarray) -> np.ndarray:
    t = x[15]
    y = np.concatenate([[t], x[:15]]).astype(np.uint32)
    y[1] ^= t
    y[3] ^= t
    y[12] ^= t
    return y


def _bs_mul(x: np.ndarray, s: int) -> np.ndarray:
    acc = x & (_M32 if s >> 15 & 1 else np.uint32(0))
    for j in range(14, -1, -1):
        acc = _bs_mulx(acc)
        if s >> j & 1:
            acc = acc ^ x
    return acc


def test_bitplane_form_matches_field():
    rng = np.random.default_rng(16)
    for _ in range(40):
        row = rng.integers(0, 256, 64, dtype=np.uint8)
        sym = to_sym(row[None])[0].astype(np.int64)
        planes = _bs_load(row)
        for p in range(16):           # plane p: bit i = symbol 2i, bit 16 + i = symbol 2i + 1
            bits = (sym >> p) & 1
            want = sum(int(bits[2 * i]) << i for i in range(16)) | sum(int(bits[2 * i + 1]) << (16 + i)
                                                                       for i in range(16))
            assert int(planes[p]) == want
        assert np.array_equal(_bs_store(planes), row)
        for s in (0, 1, 2, 0x8000, 0xFFFF, int(rng.integers(0, 65536))):
            got = to_sym(_bs_store(_bs_mul(planes, s))[None])[0]
            assert np.array_equal(got, vmul(s, sym)), s

