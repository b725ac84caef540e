"""Additive-FFT factorisation of the reference's Cauchy encode for k = 2^a.

The reference's repair coefficients are C[j][i] = inv(i ^ (k + j))
(decoder.rs:280-298).  When k is a power of two, the source points
V = {0 .. k-1} form a GF(2)-subspace of GF(2^8) and the repair points k + j
(j < r <= k) lie in its coset k + V, so

    p_j = sum_i x_i / ((k + j) + i) = R(k + j),  R(t) = N(t) / P_V(t),

with P_V(t) = prod_{v in V} (t + v) the subspace polynomial (GF(2)-linear,
P_V'(t) = Delta constant) and N = Delta * f, f the degree < k polynomial that
interpolates x over V.  P_V(k + j) = P_V(k) + P_V(j) = P_V(k), hence

    p_j = kappa * f(k + j),   kappa = Delta / P_V(k).

f is interpolated and evaluated with the Lin-Chung-Han additive FFT in the
novel polynomial basis X_i = prod_{bit q of i} W_q(t) / W_q(v_q) (W_q the
subspace polynomial of span(v_0 .. v_{q-1})): an inverse transform over V,
a fold onto the coset k + V_b (V_b = {0 .. 2^b - 1} >= the r repair points),
and a forward transform over that coset.  The GPU kernels stream the
sources in chunks of 2^c rows: each chunk is inverse-transformed in
registers, every chunk output y_m is added into two of the 2^b coset
accumulators with compile-time constants (the cross-chunk layers, the fold,
kappa and the top 2^b / 2^c forward layers, all GF(256)-linear, probed here),
and a final 2^c-point forward transform per accumulator block gives the
repairs.  Every constant is a compile-time GF(256) value, so each product is
a fixed GF(2)-linear map on bit-planes (bs_codegen).

`plan()` builds the schedule and checks it against the Cauchy matrix on
random vectors before any code is generated.
"""
from __future__ import annotations

import dataclasses
import functools
import random

# GF(2^8), poly 0x11D, generator 2 (gf_tables.rs:384-408)
_EXP = [0] * 512
_LOG = [0] * 256
_x = 1
for _i in range(255):
    _EXP[_i] = _EXP[_i + 255] = _x
    _LOG[_x] = _i
    _x <<= 1
    if _x >= 256:
        _x ^= 0x11D


def mul(a: int, b: int) -> int:
    return 0 if a == 0 or b == 0 else _EXP[_LOG[a] + _LOG[b]]


def inv(a: int) -> int:
    if a == 0:
        raise ZeroDivisionError
    return _EXP[255 - _LOG[a]]


def span_point(idx: int, basis: tuple) -> int:
    p = 0
    q = 0
    while idx:
        if idx & 1:
            p ^= basis[q]
        idx >>= 1
        q += 1
    return p


@functools.lru_cache(maxsize=None)
def _subspace_poly(b: int, t: int, basis: tuple) -> int:
    """W_b(t) = prod over span(basis[:b]) of (t + u)."""
    r = 1
    for bits in range(1 << b):
        r = mul(r, t ^ span_point(bits, basis[:b]))
    return r


def xhat(q: int, t: int, basis: tuple) -> int:
    """Normalised subspace polynomial W_q(t) / W_q(v_q) (GF(2)-linear in t)."""
    return mul(_subspace_poly(q, t, basis), inv(_subspace_poly(q, basis[q], basis)))


def mat_rows(c: int) -> list[int]:
    """Row b of the GF(2) matrix of x -> c x (bit a set iff bit b of c 2^a)."""
    cols = [mul(c, 1 << a) for a in range(8)]
    return [sum(((cols[a] >> b) & 1) << a for a in range(8)) for b in range(8)]


def macc_cost(c: int) -> int:
    """VALU ops of acc ^= c * x on 8 bit-planes with 3-input XORs."""
    if c == 0:
        return 0
    if c == 1:
        return 8
    return sum((bin(w).count("1") + 1) // 2 for w in mat_rows(c))


@dataclasses.dataclass
class Plan:
    k: int
    r: int
    ch: int                       # rows per chunk (2^c)
    R: int                        # coset accumulators (2^b >= r)
    basis: tuple
    beta_out: int
    order: list                   # load order: source index of chunk row n = hc * ch + m
    chunk_bfly: list              # per chunk: [(i, j, s)] inverse butterflies y_j ^= y_i; y_i ^= s y_j
    acc: dict                     # (hc, m) -> [(t, c)]: e_t ^= c * y_m
    final_bfly: list              # [(i, j, s)]: e_i ^= s e_j; e_j ^= e_i
    out_block: list               # repair j -> accumulator index t

    def cost(self) -> int:
        n = 0
        for bf in self.chunk_bfly:
            n += sum(8 + macc_cost(s) for _, _, s in bf)
        for hc in range(self.k // self.ch):
            for m in range(self.ch):
                for t, c in self.acc[(hc, m)]:
                    n += macc_cost(c)
        n += sum(8 + macc_cost(s) for _, _, s in self.final_bfly)
        return n

    def evaluate(self, xs: list[int]) -> list[int]:
        """The schedule on scalars (one byte per row): the r repairs."""
        e = [0] * self.R
        for hc in range(self.k // self.ch):
            y = [xs[self.order[hc * self.ch + m]] for m in range(self.ch)]
            for i, j, s in self.chunk_bfly[hc]:
                y[j] ^= y[i]
                y[i] ^= mul(s, y[j])
            for m in range(self.ch):
                for t, c in self.acc[(hc, m)]:
                    e[t] ^= mul(c, y[m])
        for i, j, s in self.final_bfly:
            e[i] ^= mul(s, e[j])
            e[j] ^= e[i]
        return [e[self.out_block[j]] for j in range(self.r)]


def transposed_evaluate(p: "Plan", t: list[int]) -> list[int]:
    """The plan run backwards with every elementary op transposed (a ^= c b
    -> b ^= c a): r repair-point values t -> the k values u_i = sum_j t_j /
    ((k + j) + i), i.e. C^T t at the plan's own op count (transposition
    principle).  The middle factor of the closed-form Cauchy inverse
    C[J,E]^-1 = diag(alpha) K diag(beta) is a sub-block of C^T; DESIGN.md 3.2
    (round 5) costs a decode solve built on it."""
    e = [0] * p.R
    for j in range(p.r):
        e[p.out_block[j]] ^= t[j]
    for i, j, s in reversed(p.final_bfly):
        e[i] ^= e[j]
        e[j] ^= mul(s, e[i])
    u = [0] * p.k
    for hc in range(p.k // p.ch):
        y = [0] * p.ch
        for m in range(p.ch):
            for tt, c in p.acc[(hc, m)]:
                y[m] ^= mul(c, e[tt])
        for i, j, s in reversed(p.chunk_bfly[hc]):
            y[j] ^= mul(s, y[i])
            y[i] ^= y[j]
        for m in range(p.ch):
            u[p.order[hc * p.ch + m]] = y[m]
    return u


def cauchy_inverse_factors(k: int, J: list[int], E: list[int]) -> tuple[list[int], list[int]]:
    """(alpha, beta) of C[J,E]^-1 = diag(alpha) K diag(beta), K[b][a] =
    1 / (x_a + y_b), x = k + J, y = E (characteristic 2: no signs)."""
    xs, e = [k + j for j in J], len(E)
    alpha, beta = [], []
    for b in range(e):
        num = den = 1
        for c in range(e):
            num = mul(num, xs[c] ^ E[b])
            if c != b:
                den = mul(den, E[b] ^ E[c])
        alpha.append(mul(num, inv(den)))
    for a in range(e):
        num = den = 1
        for c in range(e):
            num = mul(num, xs[a] ^ E[c])
            if c != a:
                den = mul(den, xs[a] ^ xs[c])
        beta.append(mul(num, inv(den)))
    return alpha, beta


def _log2(n: int) -> int:
    assert n > 0 and n & (n - 1) == 0, n
    return n.bit_length() - 1


def plan(k: int, r: int, ch: int = 8, basis: tuple | None = None, beta_out: int | None = None,
         check: int = 8) -> Plan:
    a = _log2(k)
    R = max(ch, 1 << max(0, (r - 1).bit_length()))
    b, c = _log2(R), _log2(ch)
    if not (1 <= r <= k and R <= k and c <= b and k + R <= 256):
        raise ValueError(f"no additive-FFT plan for k={k}, r={r}, ch={ch}")
    if basis is None:
        basis = tuple(1 << q for q in range(8))
    basis = tuple(basis)
    if sorted(span_point(i, basis) for i in range(R)) != list(range(R)) or \
            sorted(span_point(i, basis) for i in range(k)) != list(range(k)):
        raise ValueError("basis[:b] must span {0..2^b-1} and basis[:a] {0..k-1}")
    if beta_out is None:
        beta_out = k
    assert beta_out ^ k < R
    order = [span_point(n, basis) for n in range(k)]

    # chunk inverse transforms: layers q = 0 .. c-1 (smallest blocks first)
    chunk_bfly = []
    for hc in range(k // ch):
        bf = []
        for q in range(c):
            h = 1 << q
            for o in range(0, ch, 2 * h):
                s = xhat(q, span_point(hc * ch + o, basis), basis)
                bf += [(o + i, o + i + h, s) for i in range(h)]
        chunk_bfly.append(bf)

    delta = 1
    for u in range(1, k):
        delta = mul(delta, u)
    kappa = mul(delta, inv(_subspace_poly(a, k, basis)))
    fold = [1] * k
    for i in range(k):
        for q in range(b, a):
            if i >> q & 1:
                fold[i] = mul(fold[i], xhat(q, beta_out, basis))

    def rest(y: list[int]) -> list[int]:
        y = list(y)
        for q in range(c, a):                      # remaining inverse layers
            h = 1 << q
            for o in range(0, k, 2 * h):
                s = xhat(q, span_point(o, basis), basis)
                for i in range(o, o + h):
                    y[i + h] ^= y[i]
                    y[i] ^= mul(s, y[i + h])
        d = [0] * R
        for i in range(k):
            d[i % R] ^= mul(mul(y[i], fold[i]), kappa)
        for q in reversed(range(c, b)):            # forward layers that mix residues mod ch
            h = 1 << q
            for o in range(0, R, 2 * h):
                s = xhat(q, beta_out ^ span_point(o, basis), basis)
                for i in range(o, o + h):
                    d[i] ^= mul(s, d[i + h])
                    d[i + h] ^= d[i]
        return d

    acc = {}
    for hc in range(k // ch):
        for m in range(ch):
            y = [0] * k
            y[hc * ch + m] = 1
            d = rest(y)
            acc[(hc, m)] = [(t, d[t]) for t in range(R) if d[t]]
            assert all(t % ch == m for t, _ in acc[(hc, m)])

    final_bfly = []
    for blk in range(0, R, ch):
        for q in reversed(range(c)):
            h = 1 << q
            for o in range(blk, blk + ch, 2 * h):
                s = xhat(q, beta_out ^ span_point(o, basis), basis)
                final_bfly += [(o + i, o + i + h, s) for i in range(h)]
    out_block = [0] * r
    for t in range(R):
        j = (beta_out ^ span_point(t, basis)) ^ k
        if j < r:
            out_block[j] = t

    p = Plan(k, r, ch, R, basis, beta_out, order, chunk_bfly, acc, final_bfly, out_block)
    rng = random.Random(0x51464543)
    C = [[inv(i ^ (k + j)) for i in range(k)] for j in range(r)]
    for _ in range(check):
        xs = [rng.randrange(256) for _ in range(k)]
        ref = [0] * r
        for j in range(r):
            for i in range(k):
                ref[j] ^= mul(C[j][i], xs[i])
        if p.evaluate(xs) != ref:
            raise AssertionError("additive-FFT plan disagrees with the Cauchy matrix")
    return p


# Bases found by tools/lch_basis_search.py (lowest plane-op count of the
# schedule; any basis gives the same repairs).  Key: (k, r, ch).
BEST = {
    (64, 16, 8): ((4, 1, 11, 9, 19, 57, 64, 128), 76),     # 4,488 plane ops (canonical 5,072)
}


def best_plan(k: int, r: int, ch: int = 8) -> Plan:
    b = BEST.get((k, r, ch))
    if b is None:
        return plan(k, r, ch)
    return plan(k, r, ch, basis=b[0], beta_out=b[1])


# --------------------------------------------------------------------------
# Passes of codes the plain plan does not cover: k not a power of two, or
# repair points beyond the coset k + V (r > k or a pass j0 > 0).  The
# reference's points are x_j = k + j (integer sum, decoder.rs:280-298).  A
# pass takes the repairs whose points share one aligned coset beta + V_b
# (beta = x & ~(R - 1)); sources [0, kA), kA = 2^a the largest power of two
# <= k, go through the additive FFT evaluated on that coset (kappa and the
# fold factors taken at beta, which lies outside V_a since x >= k >= kA); the
# rows [kA, k) enter directly: each one's Cauchy column over the pass,
# pulled back through the final butterflies (an invertible linear map), is a
# set of accumulator constants like a chunk output's.
# --------------------------------------------------------------------------
def coset_passes(k: int, rt: int, R: int = 16) -> list[tuple[int, int]]:
    """(j0, r) of every pass: repairs whose points k + j share x // R."""
    out = []
    j = 0
    while j < rt:
        x = k + j
        end = min(rt, (x // R + 1) * R - k)
        out.append((j, end - j))
        j = end
    return out


@dataclasses.dataclass
class HybridPlan(Plan):
    kA: int = 0                   # rows through the FFT (plan rows 0 .. kA - 1)
    direct: dict = dataclasses.field(default_factory=dict)   # plan row n >= kA -> [(t, c)]

    def cost(self) -> int:
        n = 0
        for bf in self.chunk_bfly:
            n += sum(8 + macc_cost(s) for _, _, s in bf)
        for hc in range(self.kA // self.ch):
            for m in range(self.ch):
                n += sum(macc_cost(c) for _, c in self.acc[(hc, m)])
        for lst in self.direct.values():
            n += sum(macc_cost(c) for _, c in lst)
        n += sum(8 + macc_cost(s) for _, _, s in self.final_bfly)
        return n

    def evaluate(self, xs: list[int]) -> list[int]:
        e = [0] * self.R
        for hc in range(self.kA // self.ch):
            y = [xs[self.order[hc * self.ch + m]] for m in range(self.ch)]
            for i, j, s in self.chunk_bfly[hc]:
                y[j] ^= y[i]
                y[i] ^= mul(s, y[j])
            for m in range(self.ch):
                for t, c in self.acc[(hc, m)]:
                    e[t] ^= mul(c, y[m])
        for n, lst in self.direct.items():
            for t, c in lst:
                e[t] ^= mul(c, xs[self.order[n]])
        for i, j, s in self.final_bfly:
            e[i] ^= mul(s, e[j])
            e[j] ^= e[i]
        return [e[self.out_block[j]] for j in range(self.r)]


def hybrid_plan(k: int, rt: int, j0: int, r: int, ch: int = 8, R: int = 16, check: int = 8,
                extra_chunks: bool = True) -> HybridPlan:
    """The pass j0 .. j0 + r - 1 of the (k, rt) code (module note above).

    extra_chunks: rows [2^a, k) in whole chunks also go through a chunk
    transform, at their own points (twiddles xhat(q, i)); a chunk output's
    accumulator constants are the chunk rows' direct columns pulled through
    the chunk's inverse (computed numerically, so any invertible chunk map is
    exact; at the translated points 2^a + V_c they are as sparse as the first
    block's: 2 accumulators per output instead of 16 per direct row).  Each
    chunk is taken only where it costs fewer plane ops than its direct rows."""
    a = k.bit_length() - 1
    kA = 1 << a
    b, c = _log2(R), _log2(ch)
    x0 = k + j0
    beta = x0 & ~(R - 1)
    if not (1 <= r and j0 + r <= rt and k + rt <= 256 and (k + j0 + r - 1) & ~(R - 1) == beta and
            kA >= R and kA % ch == 0 and beta >= kA and c <= b):
        raise ValueError(f"no hybrid additive-FFT pass for k={k}, rt={rt}, j0={j0}, r={r}")
    basis = tuple(1 << q for q in range(8))
    order = list(range(k))                      # canonical basis: span_point(n) = n

    chunk_bfly = []
    for hc in range(kA // ch):
        bf = []
        for q in range(c):
            h = 1 << q
            for o in range(0, ch, 2 * h):
                s = xhat(q, hc * ch + o, basis)
                bf += [(o + i, o + i + h, s) for i in range(h)]
        chunk_bfly.append(bf)

    delta = 1
    for u in range(1, kA):
        delta = mul(delta, u)
    kappa = mul(delta, inv(_subspace_poly(a, beta, basis)))
    fold = [1] * kA
    for i in range(kA):
        for q in range(b, a):
            if i >> q & 1:
                fold[i] = mul(fold[i], xhat(q, beta, basis))

    def rest(y: list[int]) -> list[int]:
        y = list(y)
        for q in range(c, a):
            h = 1 << q
            for o in range(0, kA, 2 * h):
                s = xhat(q, o, basis)
                for i in range(o, o + h):
                    y[i + h] ^= y[i]
                    y[i] ^= mul(s, y[i + h])
        d = [0] * R
        for i in range(kA):
            d[i % R] ^= mul(mul(y[i], fold[i]), kappa)
        for q in reversed(range(c, b)):
            h = 1 << q
            for o in range(0, R, 2 * h):
                s = xhat(q, beta ^ o, basis)
                for i in range(o, o + h):
                    d[i] ^= mul(s, d[i + h])
                    d[i + h] ^= d[i]
        return d

    acc = {}
    for hc in range(kA // ch):
        for m in range(ch):
            y = [0] * kA
            y[hc * ch + m] = 1
            d = rest(y)
            acc[(hc, m)] = [(t, d[t]) for t in range(R) if d[t]]

    final_bfly = []
    for blk in range(0, R, ch):
        for q in reversed(range(c)):
            h = 1 << q
            for o in range(blk, blk + ch, 2 * h):
                s = xhat(q, beta ^ o, basis)
                final_bfly += [(o + i, o + i + h, s) for i in range(h)]
    out_block = [0] * r
    for t in range(R):
        j = (beta ^ t) - x0
        if 0 <= j < r:
            out_block[j] = t

    def final_inverse(v: list[int]) -> list[int]:
        v = list(v)
        for i, j, s in reversed(final_bfly):     # forward: v_i ^= s v_j; v_j ^= v_i
            v[j] ^= v[i]
            v[i] ^= mul(s, v[j])
        return v

    # A row's Cauchy column over the pass fixes only the r used outputs; the
    # R - r others are free.  Filling them with the column's natural values at
    # the rest of the coset, inv(i ^ (beta ^ t)) (0 where that point is row i
    # itself), keeps the pulled-back constants as sparse as a full coset's:
    # 2 accumulators per chunk output of an extra chunk instead of 3 / 9 for
    # the partial passes (12 and 15 points) of (196, 59), 24.3 k -> 16.1 k plan
    # ops for its last pass.  A direct row keeps whichever fill costs less.
    direct, natural = {}, {}
    for i in range(kA, k):
        w = [0] * R
        for j in range(r):
            w[out_block[j]] = inv(i ^ (x0 + j))
        d = final_inverse(w)
        direct[i] = [(t, d[t]) for t in range(R) if d[t]]
        w = [inv(i ^ beta ^ t) if beta ^ t != i else 0 for t in range(R)]
        d = final_inverse(w)
        natural[i] = [(t, d[t]) for t in range(R) if d[t]]
        if sum(macc_cost(c) for _, c in natural[i]) < sum(macc_cost(c) for _, c in direct[i]):
            direct[i] = natural[i]

    nA = kA
    while extra_chunks and nA + ch <= k:
        bf = []
        for q in range(c):
            h = 1 << q
            for o in range(0, ch, 2 * h):
                s = xhat(q, nA + o, basis)
                bf += [(o + i, o + i + h, s) for i in range(h)]
        cost_chunk = sum(8 + macc_cost(s) for _, _, s in bf)
        cols = {}
        for m in range(ch):
            y = [0] * ch
            y[m] = 1
            for i, j, s in reversed(bf):        # the chunk op's inverse: chunk output m -> rows
                y[i] ^= mul(s, y[j])
                y[j] ^= y[i]
            vec = [0] * R
            for ii in range(ch):
                if y[ii]:
                    for t, cc in natural[nA + ii]:
                        vec[t] ^= mul(cc, y[ii])
            cols[m] = [(t, vec[t]) for t in range(R) if vec[t]]
            cost_chunk += sum(macc_cost(cc) for _, cc in cols[m])
        if cost_chunk >= sum(macc_cost(cc) for ii in range(ch) for _, cc in direct[nA + ii]):
            break
        hc = nA // ch
        chunk_bfly.append(bf)
        for m in range(ch):
            acc[(hc, m)] = cols[m]
        for ii in range(ch):
            del direct[nA + ii]
        nA += ch

    p = HybridPlan(k, r, ch, R, basis, beta, order, chunk_bfly, acc, final_bfly, out_block, kA=nA, direct=direct)
    rng = random.Random(0x51464543 + j0)
    C = [[inv(i ^ (x0 + j)) for i in range(k)] for j in range(r)]
    for _ in range(check):
        xs = [rng.randrange(256) for _ in range(k)]
        ref = [0] * r
        for j in range(r):
            for i in range(k):
                ref[j] ^= mul(C[j][i], xs[i])
        if p.evaluate(xs) != ref:
            raise AssertionError(f"hybrid additive-FFT pass disagrees with the Cauchy matrix (k={k}, j0={j0})")
    return p
