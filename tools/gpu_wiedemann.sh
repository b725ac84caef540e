#!/bin/bash
# GPU box: k > 256 decoder timing (tools/bench_wiedemann.py) and its kernel split.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/bench_wiedemann.py --out gpurun_out/wiedemann_bench.json > gpurun_out/wiedemann.log 2>&1
rm -rf gpurun_out/prof_w8
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_w8 -o run -- python3 tools/bench_wiedemann.py --reps 1 --out gpurun_out/wiedemann_bench_prof.json > gpurun_out/wiedemann_prof.log 2>&1
python3 tools/prof_summary.py gpurun_out/prof_w8 gpurun_out/wiedemann_kernel_stats.json --command "rocprofv3 --kernel-trace --stats -- python3 tools/bench_wiedemann.py --reps 1"
echo W8_OK
