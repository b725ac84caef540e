#!/bin/bash
# GPU box: receive/send batch tests + adaptive + the C ABI test.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
    tests/test_gpu_recv_batch.py tests/test_gpu_send_batch.py tests/test_gpu_adaptive.py \
    > gpurun_out/recv_tests.log 2>&1
echo RECV_OK
