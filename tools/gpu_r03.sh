#!/bin/bash
# GPU box (round 3 iteration): encode/decode parity, one bench line, kernel stats.
#   tools/gpu_r03.sh TAG [pytest files...]
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-r03}
shift || true
OUT=gpurun_out/$TAG
mkdir -p $OUT
TESTS=${*:-tests/test_gpu_encode.py tests/test_gpu_decode.py}
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread $TESTS > $OUT/tests.log 2>&1
echo TESTS_OK
timeout -k 10 300 python bench.py --no-cpu --host-path-G 0 --c3b-G 0 --steps 10 > $OUT/bench.log 2>&1
tail -1 $OUT/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --no-cpu --host-path-G 0 --c3b-G 0 --steps 5 > $OUT/prof.log 2>&1
find $OUT/prof -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
head -8 $OUT/kernel_stats.csv
echo ALL_OK
