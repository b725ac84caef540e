#!/bin/bash
# GPU box, round 4: C5 encode passes -- one launch per pass against every pass
# in one dispatch (QF_ENCODE_MERGED), plain and additive-FFT (lch_fft.hybrid_plan)
# passes: encode / desc / C5 tests, then the C5 shapes' block + sliding encode.
#   TAG=r04s tools/gpu_r04_c5fft.sh
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-r04}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/ -m gpu \
    -x -q --timeout 170 --timeout-method thread > $OUT/c5fft_tests.log 2>&1 || { tail -30 $OUT/c5fft_tests.log; exit 1; }
tail -2 $OUT/c5fft_tests.log
SH="128,20;128,39;160,48;196,59"
for V in "0 0" "0 1" "1 0" "1 1"; do
    set -- $V
    QF_ENCODE_MERGED=$1 QF_FFT_KERNELS=$2 timeout -k 10 300 python3 tools/bench_c5.py --shapes "$SH" --modes block,sliding \
        --reps 5 --out $OUT/c5_m$1_f$2.json > $OUT/c5_m$1_f$2.log 2>&1
    echo "merged=$1 fft=$2"
    grep "^k" $OUT/c5_m$1_f$2.log
done
