#!/usr/bin/env python3
"""Summarise a `rocprofv3 --kernel-trace --stats` run into profiles/.

    python tools/prof_summary.py gpurun_out/prof profiles/r01_kernel_stats.json \
        --command "rocprofv3 ... -- python bench.py ..."

Per-kernel durations are recomputed from the kernel-trace timestamps (ns), so
the summary does not depend on the stats CSV's unit conventions; the stats CSV
itself is copied next to the JSON for reference.
"""
from __future__ import annotations

import argparse
import csv
import json
import shutil
import statistics
from collections import defaultdict
from pathlib import Path


def find(root: Path, suffix: str) -> Path | None:
    hits = sorted(root.rglob(f"*{suffix}"))
    return hits[0] if hits else None


def short(name: str) -> str:
    return name if len(name) <= 120 else name[:117] + "..."


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("prof_dir")
    ap.add_argument("out_json")
    ap.add_argument("--command", default="")
    ap.add_argument("--note", default="")
    a = ap.parse_args()
    root = Path(a.prof_dir)
    trace = find(root, "kernel_trace.csv")
    if trace is None:
        raise SystemExit(f"no kernel_trace.csv under {root}")
    dur = defaultdict(list)
    with trace.open() as f:
        for row in csv.DictReader(f):
            name = row.get("Kernel_Name") or row.get("KernelName") or "?"
            t0, t1 = int(row["Start_Timestamp"]), int(row["End_Timestamp"])
            dur[name].append((t0, t1 - t0))
    # rows of kernels on several streams are not in dispatch order: sort each
    # kernel's launches by start time, so "first" below is the earliest launch
    dur = {n: [d for _, d in sorted(v)] for n, v in dur.items()}
    total = sum(sum(v) for v in dur.values())
    kernels = []
    for name, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        kernels.append({
            "name": short(name),
            "calls": len(v),
            "avg_ms": round(statistics.mean(v) / 1e6, 4),
            "median_ms": round(statistics.median(v) / 1e6, 4),
            # the first launch of a kernel (code-object load, cold caches) aside
            "avg_after_first_ms": round(statistics.mean(v[1:]) / 1e6, 4) if len(v) > 1 else None,
            "min_ms": round(min(v) / 1e6, 4),
            "max_ms": round(max(v) / 1e6, 4),
            "total_ms": round(sum(v) / 1e6, 4),
            "pct": round(100.0 * sum(v) / total, 2),
        })
    out = {"command": a.command, "note": a.note, "source": "kernel_trace.csv (End-Start, ns)",
           "kernels": kernels}
    dst = Path(a.out_json)
    dst.parent.mkdir(parents=True, exist_ok=True)
    dst.write_text(json.dumps(out, indent=1) + "\n")
    stats = find(root, "kernel_stats.csv")
    if stats is not None:
        shutil.copy(stats, dst.with_suffix(".stats.csv"))
    for kern in kernels[:8]:
        print(f"{kern['avg_ms']:9.4f} ms x{kern['calls']:3d}  {kern['pct']:5.1f}%  {kern['name']}")


if __name__ == "__main__":
    main()
