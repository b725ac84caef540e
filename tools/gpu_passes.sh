#!/bin/bash
# GPU box: multi-pass codes with the passes on side streams (QF_PASS_STREAMS=1,
# default) vs one after the other; C5 parity tests first.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 170 --timeout-method thread tests/test_gpu_c5_mixed.py tests/test_gpu_encode.py tests/test_gpu_desc.py > $OUT/passes_tests.log 2>&1
tail -1 $OUT/passes_tests.log
SH="160,48;196,59;128,39;128,20"
QF_PASS_STREAMS=0 timeout -k 10 300 python tools/bench_c5.py --shapes "$SH" --modes block --out $OUT/c5_serial.json > $OUT/c5_serial.log 2>&1
QF_PASS_STREAMS=1 timeout -k 10 300 python tools/bench_c5.py --shapes "$SH" --modes block --out $OUT/c5_streams.json > $OUT/c5_streams.log 2>&1
QF_PASS_STREAMS=0 timeout -k 10 300 python tools/bench_c5.py --shapes "$SH" --modes block --out $OUT/c5_serial2.json > $OUT/c5_serial2.log 2>&1
QF_PASS_STREAMS=1 timeout -k 10 300 python tools/bench_c5.py --shapes "$SH" --modes block --out $OUT/c5_streams2.json > $OUT/c5_streams2.log 2>&1
python3 -c "
import json
for f in ('c5_serial', 'c5_streams', 'c5_serial2', 'c5_streams2'):
    d = json.load(open('$OUT/' + f + '.json'))
    print(f, {k: v['GiBps_alg'] for k, v in d.items() if isinstance(v, dict) and 'GiBps_alg' in v})"
