#!/usr/bin/env python3
"""Diagnostic: dump fast-path decode outputs for offline analysis."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests import oracle_py as oracle  # noqa: E402
from tests.test_gpu_decode import make_batch, run_decode  # noqa: E402
from quicfuscate_amd import fec as qf  # noqa: E402

out = {}
for (k, r, L, e) in ((16, 1, 64, 1), (16, 1, 64, 0), (16, 1, 128, 1)):
    rng = np.random.default_rng(1)
    src, gens = make_batch(oracle, rng, k, r, L, 3, k + r, erase=e, shuffle=False)
    rec, recidx, nrec, status, rrs, rec_gs = run_decode(qf, k, r, L, 3, k + r, gens, False)
    out[f"rec_{k}_{r}_{L}_{e}"] = rec
    out[f"meta_{k}_{r}_{L}_{e}"] = np.array([rrs, rec_gs])
os.makedirs("gpurun_out", exist_ok=True)
np.savez("gpurun_out/dbg2.npz", **out)
print("saved")
