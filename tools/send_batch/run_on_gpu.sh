#!/bin/bash
# GPU box: send-batch parity tests, the timing tool (M = 1, 64, 1024, with
# the per-phase host profile on stderr) and its kernel / copy trace.
# Then on the CPU side: python tools/send_batch/collect.py r02
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
rm -f gpurun_out/send_bench.jsonl gpurun_out/send_bench.err
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread \
    tests/test_gpu_send_batch.py tests/test_gpu_recv_batch.py > gpurun_out/send_tests.log 2>&1
for M in 1 64 1024; do
  QF_SEND_PROFILE=1 timeout -k 10 200 tools/send_batch/build/qf_send_bench $M >> gpurun_out/send_bench.jsonl 2>> gpurun_out/send_bench.err
done
for M in 1 64 1024; do
  timeout -k 10 200 tools/send_batch/build/qf_send_bench --recv $M >> gpurun_out/send_bench.jsonl 2>> gpurun_out/send_bench.err
done
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$R/gpurun_out/prof_send" -o send \
    -- "$R/tools/send_batch/build/qf_send_bench" 64 1024 > "$R/gpurun_out/send_prof.log" 2>&1
echo done
