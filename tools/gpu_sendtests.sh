#!/bin/bash
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/sendf
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_reference_contracts.py tests/test_gpu_send_batch.py > gpurun_out/sendf/tests2.log 2>&1 || \
    { tail -40 gpurun_out/sendf/tests2.log; exit 1; }
echo TESTS_OK
