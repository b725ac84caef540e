#!/bin/bash
# GPU box: per-packet send path parity (objects, adaptive, batches, C ABI), then its timing
# with the fused send (default) and without it (QF_SEND_FUSED=0).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/sendf
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_adaptive.py tests/test_gpu_reference_contracts.py tests/test_gpu_send_batch.py \
    tests/test_gpu_recv_batch.py tests/test_gpu_abi_c.py > gpurun_out/sendf/tests.log 2>&1 || \
    { tail -30 gpurun_out/sendf/tests.log; exit 1; }
timeout -k 10 120 tools/send_batch/build/qf_send_bench 1 64 > gpurun_out/sendf/fused.jsonl 2> gpurun_out/sendf/fused.err
QF_SEND_FUSED=0 timeout -k 10 120 tools/send_batch/build/qf_send_bench 1 64 > gpurun_out/sendf/plain.jsonl 2> gpurun_out/sendf/plain.err
echo SENDF_OK
