#!/bin/bash
# GPU box, round 4: C5 decode with the synw passes in one pass-major dispatch
# ('X') against one launch per pass (QF_ENCODE_MERGED=0).   TAG=r04ad tools/gpu_r04_c5x.sh
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-r04}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_c5_mixed.py tests/test_gpu_desc.py tests/test_gpu_decode.py \
    -x -q --timeout 170 --timeout-method thread > $OUT/c5x_tests.log 2>&1 || { tail -30 $OUT/c5x_tests.log; exit 1; }
tail -2 $OUT/c5x_tests.log
SH="${C5_SHAPES:-128,39;160,48;196,59}"
MODES="${C5_MODES:-block}"
for M in 0 1; do
    QF_ENCODE_MERGED=$M timeout -k 10 300 python3 tools/bench_c5.py --shapes "$SH" --modes $MODES \
        --reps 5 --out $OUT/c5_m$M.json > $OUT/c5_m$M.log 2>&1
    echo "merged=$M"
    grep "^k" $OUT/c5_m$M.log
done
