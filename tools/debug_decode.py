#!/usr/bin/env python3
"""Diagnostic: fast (syndrome) decode vs the general path on small scenarios."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests import oracle_py as oracle  # noqa: E402
from tests.test_gpu_decode import make_batch, run_decode  # noqa: E402
from quicfuscate_amd import fec as qf  # noqa: E402


def scenario(k, r, L, G, erase, shuffle, seed=1):
    rng = np.random.default_rng(seed)
    max_rows = k + r
    src, gens = make_batch(oracle, rng, k, r, L, G, max_rows, erase=erase, shuffle=shuffle)
    res = {}
    for path in ("fast", "general"):
        if path == "general":
            os.environ["QF_DISABLE_BS"] = "1"
        else:
            os.environ.pop("QF_DISABLE_BS", None)
        rec, recidx, nrec, status, rrs, rec_gs = run_decode(qf, k, r, L, G, max_rows, gens, False)
        bad = 0
        detail = []
        for g, (arr, rw, rc) in enumerate(gens):
            st, sol, mask = oracle.decode(k, arr, rw, None)
            erased = [i for i in range(k) if not mask[i]]
            for m, i in enumerate(erased):
                got = rec[g * rec_gs + m * rrs: g * rec_gs + m * rrs + L]
                if not (got == src[g, i]).all():
                    bad += 1
                    nb = int((got != src[g, i]).sum())
                    first = int(np.argmax(got != src[g, i]))
                    C = oracle.cauchy(k, r)
                    detail.append((g, m, i, nb, first, got[:6].tolist(), src[g, i, :6].tolist()))
        res[path] = (bad, detail[:4], list(status[:4]), list(nrec[:4]))
    os.environ.pop("QF_DISABLE_BS", None)
    print(f"k={k} r={r} L={L} G={G} e={erase} shuffle={shuffle}: fast={res['fast']} general_bad={res['general'][0]}",
          flush=True)


if __name__ == "__main__":
    for (k, r) in ((16, 1), (16, 16), (64, 16)):
        for L in (64, 1200):
            for e in sorted({1, 2, min(k, r)}):
                if e > r:
                    continue
                for sh in (False, True):
                    scenario(k, r, L, 3, e, sh)
