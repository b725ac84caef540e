#!/bin/bash
# GPU box, round 4: decode / desc / C5 tests, then the C5 mixed desc batch
# with the pass-major dispatches (QF_ENCODE_MERGED=1) and without.
#   TAG=r04af tools/gpu_r04_c5pm.sh
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-r04}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests/test_gpu_c5_mixed.py tests/test_gpu_desc.py tests/test_gpu_decode.py \
    tests/test_gpu_recv_batch.py -x -q --timeout 170 --timeout-method thread > $OUT/pm_tests.log 2>&1 || { tail -30 $OUT/pm_tests.log; exit 1; }
tail -2 $OUT/pm_tests.log
for M in 0 1; do
    QF_ENCODE_MERGED=$M timeout -k 10 300 python3 tools/bench_c5.py --mixed-only --reps 3 \
        --out $OUT/mixed_m$M.json > $OUT/mixed_m$M.log 2>&1
    python3 -c "import json; d=json.load(open('$OUT/mixed_m$M.json'))['mixed_desc_batch']; print('merged=$M', d['round_trip_ok'], d['encode']['GiBps_alg'], d['decode']['GiBps_alg'], {n: round(v[1], 3) for n, v in d['decode']['kernels'].items()})"
done
