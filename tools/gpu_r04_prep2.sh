#!/bin/bash
# GPU box: the per-lane acceptance pass's tests and the bench line serial / split.
#   TAG=r04o tools/gpu_r04_prep2.sh
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-r04}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py -k "per_lane or bench_shape or duplicates" tests/test_gpu_fullsize.py -x -q --timeout 170 --timeout-method thread > $OUT/dec_tests.log 2>&1 || { tail -30 $OUT/dec_tests.log; exit 1; }
tail -1 $OUT/dec_tests.log
ARGS="--no-cpu --host-path-G 0 --c3b-G 0 --c4-G 0 --c5-mixed-bytes 0 --steps 20"
for mode in serial split; do
  flag=""; [ $mode = serial ] && flag="--serial"
  timeout -k 10 200 python3 bench.py $ARGS $flag > $OUT/bench_${mode}.log 2>&1
  python3 -c "
import json
d=json.loads(open('$OUT/bench_${mode}.log').read().strip().splitlines()[-1])
print('$mode', d['value'], d['ms_per_step'], d['kernel_ms_per_launch'], d['roofline_encode']['launch_ms'])"
done
