#!/bin/bash
# GPU box: codec parity (encode, decode, C5, desc, full size) then one bench line.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/quick
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_encode.py tests/test_gpu_decode.py tests/test_gpu_c5_mixed.py tests/test_gpu_desc.py \
    tests/test_gpu_fullsize.py > gpurun_out/quick/tests.log 2>&1
timeout -k 10 300 python bench.py --no-cpu --host-path-G 0 > gpurun_out/quick/bench.log 2>&1
echo QUICK_OK
