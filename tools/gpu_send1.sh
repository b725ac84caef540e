#!/bin/bash
# GPU box: per-packet send path (M = 1) timing and its kernel / copy trace.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/send1
timeout -k 10 120 tools/send_batch/build/qf_send_bench 1 > gpurun_out/send1/bench.jsonl 2> gpurun_out/send1/bench.err
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$R/gpurun_out/send1/prof" -o send \
    -- "$R/tools/send_batch/build/qf_send_bench" 1 > "$R/gpurun_out/send1/prof.log" 2>&1
echo SEND1_OK
