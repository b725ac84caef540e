#!/bin/bash
# GPU box: GF(2^16) tests (FFT encode first) and the GF(2^16) bench.
#   TAG=r03ac tools/gpu_fft16.sh
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-r03}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_gf16.py -x -v --timeout 120 --timeout-method thread -k "fft" > $OUT/fft_tests.log 2>&1
tail -3 $OUT/fft_tests.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_gf16.py -x -q --timeout 170 --timeout-method thread > $OUT/gf16_tests.log 2>&1 || { tail -30 $OUT/gf16_tests.log; exit 1; }
tail -2 $OUT/gf16_tests.log
timeout -k 10 300 python tools/bench_gf16.py --out $OUT/gf16_bench.json > $OUT/gf16_bench.log 2>&1
tail -12 $OUT/gf16_bench.log
