#!/bin/bash
# GPU box, round 4: C5 decode with the additive-FFT synw passes ('V') against
# the plain passes (QF_FFT_KERNELS=0 also takes the plain merged encode).
#   TAG=r04ac tools/gpu_r04_c5v.sh
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-r04}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_c5_mixed.py tests/test_gpu_desc.py tests/test_gpu_decode.py \
    -x -q --timeout 170 --timeout-method thread > $OUT/c5v_tests.log 2>&1 || { tail -30 $OUT/c5v_tests.log; exit 1; }
tail -2 $OUT/c5v_tests.log
SH="128,39;160,48;196,59"
for F in 0 1; do
    QF_FFT_KERNELS=$F timeout -k 10 300 python3 tools/bench_c5.py --shapes "$SH" --modes block \
        --reps 5 --out $OUT/c5_f$F.json > $OUT/c5_f$F.log 2>&1
    echo "fft=$F"
    grep "^k" $OUT/c5_f$F.log
done
