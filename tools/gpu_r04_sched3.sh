#!/bin/bash
# GPU box, round 4: bench step schedules alternating on one box: payload
# stream (default), serial, payload stream with a 2-block-per-CU acceptance grid.
#   TAG=r04ak tools/gpu_r04_sched3.sh
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-r04}
OUT=gpurun_out/$TAG
mkdir -p $OUT
ARGS="--steps 20 --warmup 5 --no-cpu --host-path-G 0 --c3b-G 0 --c4-G 0 --c5-mixed-bytes 0"
for i in 1 2 3; do
  for V in "default" "serial" "grid512"; do
    case $V in
      default) E=""; F="";;
      serial) E=""; F="--serial";;
      grid512) E="QF_PREPARE_GRID=512"; F="";;
    esac
    env $E timeout -k 10 200 python3 bench.py $ARGS $F > $OUT/b.log 2>&1
    python3 -c "import json; d=json.loads(open('$OUT/b.log').read().strip().splitlines()[-1]); print('$V', d['value'], d['ms_per_step'], d['ms_per_step_median_rank0'], d['encode_ms'], d['decode_ms'], d['verified'])" | tee -a $OUT/sched3.txt
  done
done
