#!/bin/bash
# GPU box: GF(2^16) parity + throughput (bit-sliced encode, round 3).
#   TAG=r03x tools/gpu_gf16.sh
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-r03}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 170 --timeout-method thread tests/test_gpu_gf16.py tests/test_gpu_adaptive.py > $OUT/gf16_tests.log 2>&1
tail -2 $OUT/gf16_tests.log
timeout -k 10 300 python tools/bench_gf16.py --out $OUT/gf16_bench.json > $OUT/gf16_bench.log 2>&1
timeout -k 10 300 python tools/bench_gf16.py --G 65536 --reps 3 --out $OUT/gf16_bench_G65536.json > $OUT/gf16_bench65536.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/gf16_kt -o run -- python3 tools/bench_gf16.py --reps 3 --out $OUT/gf16_bench_prof.json > $OUT/gf16_kt.log 2>&1
find $OUT/gf16_kt -name '*kernel_stats.csv' -exec cp {} $OUT/gf16_kernel_stats.csv \;
head -12 $OUT/gf16_kernel_stats.csv | cut -c1-200
echo GF16_OK
