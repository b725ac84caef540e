#!/bin/bash
# GPU box: bit-sliced payload pass (k_combine_bs) parity, then C5 decode timing
# with it (default) and without it (QF_COMBINE_BS=0).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/cbs
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_decode.py tests/test_gpu_c5_mixed.py tests/test_gpu_desc.py > gpurun_out/cbs/tests.log 2>&1
SH="${C5_SHAPES:-32,5;128,20;196,59}"
timeout -k 10 300 python3 tools/bench_c5.py --shapes "$SH" --modes block --reps 5 \
    --out gpurun_out/cbs/bs.json > gpurun_out/cbs/bs.log 2>&1
QF_COMBINE_BS=0 timeout -k 10 300 python3 tools/bench_c5.py --shapes "$SH" --modes block --reps 5 \
    --out gpurun_out/cbs/slots.json > gpurun_out/cbs/slots.log 2>&1
echo CBS_OK
