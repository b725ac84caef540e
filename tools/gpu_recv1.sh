#!/bin/bash
# GPU box: decoder object / receive parity, then per-packet and batch receive timing.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/recv1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_reference_contracts.py tests/test_gpu_recv_batch.py tests/test_gpu_adaptive.py \
    tests/test_gpu_abi_c.py > gpurun_out/recv1/tests.log 2>&1 || { tail -40 gpurun_out/recv1/tests.log; exit 1; }
timeout -k 10 200 tools/send_batch/build/qf_send_bench --recv 1 64 1024 > gpurun_out/recv1/recv.jsonl 2> gpurun_out/recv1/recv.err
echo RECV1_OK
