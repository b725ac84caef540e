#!/bin/bash
# GPU box: the default bench line (split C4 leg) and a serial one, for the C4 schedule comparison.
#   TAG=r03ab tools/gpu_c4.sh
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-r03}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python bench.py > $OUT/bench_split.log 2>&1
tail -1 $OUT/bench_split.log | cut -c1-300
timeout -k 10 400 python bench.py --serial > $OUT/bench_serial.log 2>&1
tail -1 $OUT/bench_serial.log | cut -c1-300
timeout -k 10 300 python -u -m pytest tests/test_gpu_bench_ranks.py -x -q --timeout 250 --timeout-method thread > $OUT/ranks.log 2>&1
tail -2 $OUT/ranks.log
