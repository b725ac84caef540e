#!/bin/bash
# GPU box: send-batch tests, per-phase host timing (QF_SEND_PROFILE) and the
# kernel trace of the timing tool.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_send_batch.py > gpurun_out/send_tests.log 2>&1
B=tools/send_batch/build/qf_send_bench
for ch in 1 2 4; do
  echo "chunks $ch" >> gpurun_out/sp.log
  QF_SEND_CHUNKS=$ch QF_SEND_PROFILE=1 timeout -k 10 120 $B 1024 >> gpurun_out/sp.log 2>&1
done
for th in 0 3 7; do
  echo "threads $th" >> gpurun_out/sp.log
  QF_COPY_THREADS=$th QF_SEND_PROFILE=1 timeout -k 10 120 $B 1024 >> gpurun_out/sp.log 2>&1
done
