#!/usr/bin/env python3
"""SQ counters of the C5 sliding-window encode launches (tools/gpu.sh c5sq)
-> profiles/c5_sq_counters.json, keyed "<mode>/<kernel>/G<G>" with per-launch
means and the code hash of the kernel measured (bench_c5._valu_info reads
them only while the built kernel has that hash).

    python tools/c5_sq_summary.py <pmc dir> <bench_c5 json> --mode sliding --out profiles/c5_sq_counters.json
"""
import argparse
import csv
import json
from collections import defaultdict
from pathlib import Path

ap = argparse.ArgumentParser()
ap.add_argument("pmc")
ap.add_argument("bench", help="bench_c5.py --out of the same command (G and kernels per shape)")
ap.add_argument("--mode", default="sliding")
ap.add_argument("--out", required=True)
ap.add_argument("--command", default="")
a = ap.parse_args()
acc = defaultdict(float)
for fp in sorted(Path(a.pmc).rglob("*counter_collection.csv")):
    with fp.open() as f:
        for row in csv.DictReader(f):
            name = row.get("Kernel_Name", "?").split("(")[0].strip()
            if not name.startswith("qf_"):
                continue
            acc[(name, row["Dispatch_Id"], row["Counter_Name"])] += float(row["Counter_Value"])
per = defaultdict(lambda: defaultdict(list))
for (name, _, ctr), v in acc.items():
    per[name][ctr].append(v)
bench = json.loads(Path(a.bench).read_text())
root = Path(__file__).resolve().parents[1]
hashes = json.loads((root / "quicfuscate_amd" / "lib" / "kernel_hashes.json").read_text())
out = {"_command": a.command,
       "_note": "per-launch means over the launches of the counter pass (warm-up and timed reps alike); "
                "SQ_BUSY_CYCLES / SQ_WAVE_CYCLES in quad-cycles (MI355X_MICROARCH.md)"}
prev = Path(a.out)
if prev.exists():   # other modes / shapes of earlier passes stay
    out.update({k: v for k, v in json.loads(prev.read_text()).items() if not k.startswith("_")})
for key, v in bench.items():
    if not key.startswith("k") or f"{a.mode}/encode" not in v:
        continue
    ent = v[f"{a.mode}/encode"]
    for name in ent["kernels"]:
        if name not in per:
            continue
        d = {c: sum(x) / len(x) for c, x in sorted(per[name].items())}
        d["launches"] = len(next(iter(per[name].values())))
        d["code_sha16"] = hashes.get(name)
        if d.get("SQ_WAVES"):
            d["valu_per_wave"] = round(d["SQ_INSTS_VALU"] / d["SQ_WAVES"], 1)
        out[f"{a.mode}/{name}/G{ent['G']}"] = d
Path(a.out).write_text(json.dumps(out, indent=1))
print(json.dumps({k: v.get("valu_per_wave") for k, v in out.items() if not k.startswith("_")}, indent=1))
