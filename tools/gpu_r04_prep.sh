#!/bin/bash
# GPU box, round 4: decode tests with the per-lane acceptance pass, then the
# bench line serial and split, each with the per-lane and per-wave pass.
#   TAG=r04l tools/gpu_r04_prep.sh
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-r04}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_fullsize.py -x -q --timeout 170 --timeout-method thread > $OUT/dec_tests.log 2>&1 || { tail -30 $OUT/dec_tests.log; exit 1; }
tail -2 $OUT/dec_tests.log
ARGS="--no-cpu --host-path-G 0 --c3b-G 0 --c4-G 0 --c5-mixed-bytes 0 --steps 20"
for mode in serial split; do
  for lanes in 1 0; do
    flag=""; [ $mode = serial ] && flag="--serial"
    QF_PREPARE_LANES=$lanes timeout -k 10 200 python3 bench.py $ARGS $flag > $OUT/bench_${mode}_l$lanes.log 2>&1
    python3 -c "
import json,sys
d=json.loads(open('$OUT/bench_${mode}_l$lanes.log').read().strip().splitlines()[-1])
print('$mode lanes=$lanes', d['value'], d['ms_per_step'], d['kernel_ms_per_launch'], d['roofline_encode']['launch_ms'])"
  done
done
