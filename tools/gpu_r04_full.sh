#!/bin/bash
# GPU box, round 4: the whole -m gpu suite, smoke, one default bench line
# (with the c5 leg).   TAG=r04c tools/gpu_r04_full.sh
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-r04}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 840 python -u -m pytest tests -m gpu -x -q --timeout 170 --timeout-method thread > $OUT/gpu_tests.log 2>&1
tail -3 $OUT/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $OUT/smoke.log 2>&1
tail -1 $OUT/smoke.log
timeout -k 10 400 python bench.py > $OUT/bench_full.log 2>&1
tail -1 $OUT/bench_full.log | cut -c1-400
if [ "${WITH_LAB:-0}" = "1" ]; then
  timeout -k 10 240 python3 tools/dec_lab.py run --reps 10 --out $OUT/dec_lab.json > $OUT/dec_lab.log 2>&1
  echo DEC_LAB_OK
fi
