#!/bin/bash
# GPU box, round 4: hybrid plans with the rows past 2^a in transformed chunks
# (encode 'N', pass-major FFT synw 'Y') against the plain passes (QF_FFT_KERNELS=0:
# 'M' encode, 'X' synw): encode / decode / desc / C5 tests, then the C5 shapes.
#   TAG=r04al tools/gpu_r04_c5y.sh
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-r04}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 800 python -u -m pytest tests/test_gpu_c5_mixed.py tests/test_gpu_desc.py tests/test_gpu_decode.py \
    tests/test_gpu_encode.py -x -q --timeout 170 --timeout-method thread > $OUT/y_tests.log 2>&1 || { tail -30 $OUT/y_tests.log; exit 1; }
tail -2 $OUT/y_tests.log
SH="128,39;160,48;196,59"
for F in 0 1; do
    QF_FFT_KERNELS=$F timeout -k 10 300 python3 tools/bench_c5.py --shapes "$SH" --modes block,sliding \
        --reps 5 --out $OUT/c5_f$F.json > $OUT/c5_f$F.log 2>&1
    echo "fft=$F"
    grep "^k" $OUT/c5_f$F.log
done
QF_FFT_KERNELS=1 timeout -k 10 300 python3 tools/bench_c5.py --mixed-only --reps 3 --out $OUT/mixed.json > $OUT/mixed.log 2>&1
python3 -c "import json; d=json.load(open('$OUT/mixed.json'))['mixed_desc_batch']; print('mixed', d['round_trip_ok'], d['encode']['GiBps_alg'], d['decode']['GiBps_alg'])"
