#!/usr/bin/env python3
"""Per-kernel means of rocprofv3 --pmc counters (counter_collection.csv).

    python tools/sq_summary.py gpurun_out/pmc_sq [out.json]"""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

root = Path(sys.argv[1])
acc = defaultdict(float)
for fp in sorted(root.rglob("*counter_collection.csv")):
    with fp.open() as f:
        for row in csv.DictReader(f):
            acc[(row.get("Kernel_Name", "?"), row.get("Dispatch_Id", "?"), row["Counter_Name"])] += float(row["Counter_Value"])
per = defaultdict(lambda: defaultdict(list))
for (name, disp, ctr), v in acc.items():
    per[name[:60]][ctr].append(v)
out = {n: {c: sum(v) / len(v) for c, v in sorted(d.items())} for n, d in per.items()}
# the code object each entry measured (generated kernels; bench.py uses the
# counters only while the built kernel has the same hash)
hfile = Path(__file__).resolve().parents[1] / "quicfuscate_amd" / "lib" / "kernel_hashes.json"
hashes = json.loads(hfile.read_text()) if hfile.exists() else {}
for n in out:
    h = next((v for kname, v in hashes.items() if n == kname or n.startswith(kname)), None)
    if h:
        out[n]["code_sha16"] = h
print(json.dumps(out, indent=1))
if len(sys.argv) > 2:
    Path(sys.argv[2]).write_text(json.dumps(out, indent=1))
