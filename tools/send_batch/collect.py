"""Collects a send-batch GPU run (tools/send_batch/run_on_gpu.sh) into
profiles/<tag>_on_send_batch.json and copies the kernel/copy stats next to it."""
import csv
import json
import shutil
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[2]
OUT = REPO / "gpurun_out"


def main(tag: str) -> None:
    rows = [json.loads(l) for l in (OUT / "send_bench.jsonl").read_text().splitlines() if l.startswith("{")]
    phases = [l for l in (OUT / "send_bench.err").read_text().splitlines() if l.startswith("[qf send batch]")]
    stats = {}
    for name in ("send_kernel_stats.csv", "send_memory_copy_stats.csv"):
        src = OUT / "prof_send" / name
        dst = REPO / "profiles" / f"{tag}_on_send_batch_{name.replace('send_', '')}"
        shutil.copy(src, dst)
        stats[name] = [{k: r[k] for k in ("Name", "Calls", "AverageNs")} for r in csv.DictReader(open(src))]
    doc = {
        "what": "AdaptiveFec.on_send over M connections (Normal mode, k=64, n=74, 1200-byte packets, full "
                "windows: 10 repairs per packet); host wall clock per source packet.  Rows with leg=receive: "
                "on_receive of one generation per connection (58 of 64 sources + 10 repairs), per packet",
        "tool": "tools/send_batch/qf_send_bench.c (run_on_gpu.sh)",
        "batch": "qf_adaptive_on_send_batch / qf_adaptive_on_receive_batch: one call per round of M packets",
        "sequential": "qf_adaptive_on_send per packet (the per-connection path)",
        "results": rows,
        "phase_profile_us_per_call": phases,
        "rocprof_stats_M64_and_M1024_run": stats,
    }
    (REPO / "profiles" / f"{tag}_on_send_batch.json").write_text(json.dumps(doc, indent=1) + "\n")
    print(json.dumps(rows, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r02")
