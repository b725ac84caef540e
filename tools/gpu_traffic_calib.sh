#!/bin/bash
# GPU box: FETCH_SIZE calibration of the fused decode's gather (tools/traffic_calib.py).
# Needs the calibration manifest: python3 tools/dec_lab.py build --calib (in the container).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03}/calib
mkdir -p $OUT
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 tools/dec_lab.py run --reps 3 --out $OUT/lab_f.json > $OUT/fetch.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 tools/dec_lab.py run --reps 3 --out $OUT/lab_w.json > $OUT/write.log 2>&1
python3 tools/traffic_calib.py $OUT/fetch $OUT/write --out $OUT/traffic_calib.json
echo CALIB_OK
