#!/bin/bash
# GPU box, round 4: single-pass hybrid FFT encode ('E') for (96, 15) / (48, 8)
# against the plain kernels (QF_FFT_KERNELS=0).   TAG=r04an tools/gpu_r04_c5e.sh
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-r04}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_encode.py tests/test_gpu_desc.py tests/test_gpu_c5_mixed.py \
    -x -q --timeout 170 --timeout-method thread > $OUT/e_tests.log 2>&1 || { tail -30 $OUT/e_tests.log; exit 1; }
tail -2 $OUT/e_tests.log
for F in 0 1; do
    QF_FFT_KERNELS=$F timeout -k 10 300 python3 tools/bench_c5.py --shapes "96,15;48,8" --modes block,sliding \
        --reps 5 --out $OUT/c5_f$F.json > $OUT/c5_f$F.log 2>&1
    echo "fft=$F"
    grep "^k" $OUT/c5_f$F.log
done
