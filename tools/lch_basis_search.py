#!/usr/bin/env python3
"""Search the subspace basis (and the output coset representative) of the
additive-FFT encode plan (quicfuscate_amd/lch_fft.py) for the lowest
plane-op count.  Every basis gives the same repairs; the constants, and so
the XOR count of each bit-sliced product, differ.

  python tools/lch_basis_search.py --k 64 --r 16 --ch 8 --iters 3000

Prints the best (basis, beta_out) found; lch_fft.BEST holds the results."""
from __future__ import annotations

import argparse
import random
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from quicfuscate_amd import lch_fft as L  # noqa: E402


def valid(basis, a, b):
    return (sorted(L.span_point(i, basis) for i in range(1 << b)) == list(range(1 << b))
            and sorted(L.span_point(i, basis) for i in range(1 << a)) == list(range(1 << a)))


def mutate(rng, basis, beta, a, b, k):
    basis = list(basis)
    kind = rng.randrange(4)
    if kind == 0 and b > 1:          # v_i ^= v_j inside the repair subspace
        i, j = rng.sample(range(b), 2)
        basis[i] ^= basis[j]
    elif kind == 1 and a > b:        # upper vector += anything
        i = rng.randrange(b, a)
        j = rng.choice([q for q in range(a) if q != i])
        basis[i] ^= basis[j]
    elif kind == 2:                  # swap inside a level
        lo, hi = (0, b) if rng.random() < 0.5 or a - b < 2 else (b, a)
        if hi - lo >= 2:
            i, j = rng.sample(range(lo, hi), 2)
            basis[i], basis[j] = basis[j], basis[i]
    else:
        beta = k ^ rng.randrange(1 << b)
    return tuple(basis), beta


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=64)
    ap.add_argument("--r", type=int, default=16)
    ap.add_argument("--ch", type=int, default=8)
    ap.add_argument("--iters", type=int, default=2000)
    ap.add_argument("--seed", type=int, default=1)
    args = ap.parse_args()
    k, r, ch = args.k, args.r, args.ch
    p0 = L.plan(k, r, ch, check=1)
    a, b = k.bit_length() - 1, p0.R.bit_length() - 1
    rng = random.Random(args.seed)
    best = (p0.cost(), p0.basis, p0.beta_out)
    cur = best
    print("canonical", best[0], flush=True)
    for it in range(args.iters):
        if rng.random() < 0.02:      # restart from the best
            cur = best
        nb, nbeta = mutate(rng, cur[1], cur[2], a, b, k)
        if not valid(nb, a, b):
            continue
        c = L.plan(k, r, ch, basis=nb, beta_out=nbeta, check=0).cost()
        if c <= cur[0] or rng.random() < 0.05:
            cur = (c, nb, nbeta)
        if c < best[0]:
            best = (c, nb, nbeta)
            print(it, best, flush=True)
    L.plan(k, r, ch, basis=best[1], beta_out=best[2], check=16)   # verified
    print("best", best)


if __name__ == "__main__":
    main()
