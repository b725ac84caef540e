#!/usr/bin/env python3
"""FETCH_SIZE calibration for the fused decode's access pattern (VERDICT r02
item 3; MI355X_MICROARCH.md HBM section: FETCH_SIZE is calibrated only for
wide streaming reads, "calibrate on a known byte count in your own access
pattern").

    rocprofv3 --pmc FETCH_SIZE -d D1 -- python3 tools/dec_lab.py run   (calibration manifest)
    rocprofv3 --pmc WRITE_SIZE -d D2 -- python3 tools/dec_lab.py run
    python tools/traffic_calib.py D1 D2 --out profiles/traffic_calib.json

dec_calib_reads is the library's decode kernel with the LU and the stores
stripped: per generation it reads 64 rows of L bytes (51 surviving sources
and 13 repairs, through the slot map), the slot map (80 B) and the record's
rank quad (16 B) from HBM; its 13 zero-row reads hit L2.  factor = those
bytes / FETCH_SIZE bytes; the full kernel's HBM traffic = FETCH x factor +
WRITE_SIZE (exact for 16-B-per-lane stores per the guide)."""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from pmc_traffic import per_dispatch  # noqa: E402


def mean_of(d: dict, stem: str) -> float:
    vals = [v for n, vs in d.items() if stem in n for v in vs]
    if not vals:
        raise SystemExit(f"no dispatch of {stem}")
    return sum(vals) / len(vals)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--G", type=int, default=65536)
    ap.add_argument("--k", type=int, default=64)
    ap.add_argument("--e", type=int, default=13)
    ap.add_argument("--L", type=int, default=1200)
    ap.add_argument("--out", default="profiles/traffic_calib.json")
    a = ap.parse_args()
    fetch = per_dispatch(Path(a.fetch_dir), "FETCH_SIZE")
    write = per_dispatch(Path(a.write_dir), "WRITE_SIZE")
    known = a.G * (a.k * a.L + 80 + 16)
    raw_calib = mean_of(fetch, "dec_calib_reads") * 1024
    factor = known / raw_calib
    full_fetch = mean_of(fetch, "dec_calib_full") * 1024
    full_write = mean_of(write, "dec_calib_full") * 1024
    calib_write = mean_of(write, "dec_calib_reads") * 1024
    alg = a.G * ((a.k + a.e) * a.L + 80 + 272)
    out = {"kernel": "fused decode (library 'C' kernel, lab build dec_calib_full)",
           "known_read_bytes_calib_kernel": known, "fetch_size_bytes_calib_kernel": raw_calib,
           "fetch_factor": round(factor, 4), "write_size_bytes_calib_kernel": calib_write,
           "full_fetch_size_bytes": full_fetch, "full_write_bytes": full_write,
           "full_hbm_bytes_calibrated": round(full_fetch * factor + full_write),
           "algorithmic_bytes": alg,
           "calibrated_over_algorithmic": round((full_fetch * factor + full_write) / alg, 4),
           "note": "factor from the same kernel stripped to its reads (known bytes, same gather); "
                   "the guide's streaming-read factor is 2"}
    Path(a.out).write_text(json.dumps(out, indent=1))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
