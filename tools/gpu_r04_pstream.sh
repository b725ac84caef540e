#!/bin/bash
# GPU box, round 4: payload-stream decode tests, then the bench step with the
# decode's payload pass on the encode's stream (--payload-stream) against the
# default split schedule, alternating, 3 runs each.   TAG=r04ah tools/gpu_r04_pstream.sh
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-r04}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py -x -q --timeout 170 --timeout-method thread \
    -k "payload" > $OUT/ps_tests.log 2>&1 || { tail -30 $OUT/ps_tests.log; exit 1; }
tail -2 $OUT/ps_tests.log
ARGS="--steps 20 --warmup 5 --no-cpu --host-path-G 0 --c3b-G 0 --c4-G 0 --c5-mixed-bytes 0"
for i in 1 2 3; do
  for V in "--cross-stream" ""; do
    timeout -k 10 200 python3 bench.py $ARGS $V > $OUT/b.log 2>&1
    python3 -c "import json; d=json.loads(open('$OUT/b.log').read().strip().splitlines()[-1]); print('$V' or 'payload-stream', d['value'], d['ms_per_step'], d['ms_per_step_median_rank0'], d['encode_ms'], d['decode_ms'], d['verified'])" | tee -a $OUT/sched.txt
  done
done
