#!/bin/bash
# GPU box: send-batch tests (bursts of one connection in one call) and the
# native per-packet driver.   TAG=r04g tools/gpu_r04_burst.sh
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-r04}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_send_batch.py tests/test_gpu_adaptive.py -x -v --timeout 170 --timeout-method thread > $OUT/send_tests.log 2>&1 || { tail -40 $OUT/send_tests.log; exit 1; }
tail -3 $OUT/send_tests.log
timeout -k 10 200 tools/send_batch/build/bench_on_send 300 > $OUT/on_send_native.json 2> $OUT/on_send_native.err
python3 -c "import json; d=json.load(open('$OUT/on_send_native.json')); print(json.dumps(d['batch1']))"
