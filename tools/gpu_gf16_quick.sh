#!/bin/bash
# GPU box: GF(2^16) bit-sliced parity + batched throughput (encode and decode).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 170 --timeout-method thread tests/test_gpu_gf16.py > $OUT/gf16q_tests.log 2>&1
tail -1 $OUT/gf16q_tests.log
timeout -k 10 300 python tools/bench_gf16.py --out $OUT/gf16q_bench.json > $OUT/gf16q_bench.log 2>&1
timeout -k 10 300 python tools/bench_gf16.py --G 65536 --reps 3 --out $OUT/gf16q_bench65536.json > $OUT/gf16q_bench65536.log 2>&1
python3 -c "
import json
for f in ('$OUT/gf16q_bench.json', '$OUT/gf16q_bench65536.json'):
    d = json.load(open(f))
    for kk in ('batched_k64_r16/encode16', 'batched_k64_r16/decode16'):
        v = d[kk]; print(f, kk, v['G'], v['GiBps_alg'], v['kernels'])"
