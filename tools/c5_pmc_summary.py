#!/usr/bin/env python3
"""Per-kernel averages of rocprofv3 --pmc runs (counter_collection.csv) for
the C5 pass kernels: FETCH_SIZE doubled per MI355X_MICROARCH.md (gfx950 counts
half the bytes of a wide streaming read), SQ counters as is.

    python tools/c5_pmc_summary.py <pmc dir> [<pmc dir> ...] --out gpurun_out/x.json
"""
import argparse
import csv
import json
from collections import defaultdict
from pathlib import Path

ap = argparse.ArgumentParser()
ap.add_argument("dirs", nargs="+")
ap.add_argument("--out", required=True)
ap.add_argument("--match", default="qf_,k_", help="comma-separated substrings a kernel name must contain (any)")
a = ap.parse_args()
match = [m for m in a.match.split(",") if m]
acc = defaultdict(float)
for d in a.dirs:
    for fp in sorted(Path(d).rglob("*counter_collection.csv")):
        with fp.open() as f:
            for row in csv.DictReader(f):
                name = row.get("Kernel_Name", "?")
                if not any(m in name for m in match):
                    continue
                acc[(name.split("(")[0].strip(), row["Dispatch_Id"], row["Counter_Name"])] += float(row["Counter_Value"])
per = defaultdict(lambda: defaultdict(list))
for (name, _, ctr), v in acc.items():
    per[name][ctr].append(v)
res = {}
for name, ctrs in per.items():
    res[name] = {c: sum(v) / len(v) for c, v in ctrs.items()}
    if "FETCH_SIZE" in res[name]:
        res[name]["fetch_bytes_corrected"] = res[name]["FETCH_SIZE"] * 1024 * 2
    if "WRITE_SIZE" in res[name]:
        res[name]["write_bytes"] = res[name]["WRITE_SIZE"] * 1024
    print(name, {c: round(x, 1) for c, x in res[name].items()}, flush=True)
Path(a.out).write_text(json.dumps(res, indent=1))
