#!/bin/bash
# GPU box: C5 decode parity (c5_mixed, desc batches) then the C5 bench.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
    tests/test_gpu_c5_mixed.py tests/test_gpu_desc.py > gpurun_out/c5_tests.log 2>&1
timeout -k 10 500 python3 tools/bench_c5.py --out gpurun_out/c5_bench.json > gpurun_out/c5.log 2>&1
echo C5_OK
