#!/bin/bash
# GPU box, round 4: rocprofv3 kernel trace of the default bench step (and of
# the serial schedule), summarised per kernel.   TAG=r04aj tools/gpu_r04_kt.sh
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-r04}
OUT=gpurun_out/$TAG
mkdir -p $OUT
ARGS="--steps 10 --warmup 3 --no-cpu --host-path-G 0 --c3b-G 0 --c4-G 0 --c5-mixed-bytes 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 bench.py $ARGS > $OUT/kt.log 2>&1
grep '^{"metric"' $OUT/kt.log > $OUT/kt.bench.json
python3 tools/prof_summary.py $OUT/kt $OUT/kernel_stats.json --command "rocprofv3 --kernel-trace --stats --output-format csv -- python3 bench.py $ARGS"
echo KT_OK
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kts -o run -- python3 bench.py $ARGS --serial > $OUT/kts.log 2>&1
python3 tools/prof_summary.py $OUT/kts $OUT/kernel_stats_serial.json --command "rocprofv3 --kernel-trace --stats --output-format csv -- python3 bench.py $ARGS --serial"
echo KTS_OK
