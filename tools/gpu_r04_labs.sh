#!/bin/bash
# GPU box: the encode and decode labs as built (tools/bs_lab.py build, tools/dec_lab.py build).
#   TAG=r04d tools/gpu_r04_labs.sh
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-r04d}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 240 python3 tools/dec_lab.py run --reps 10 --out $OUT/dec_lab.json > $OUT/dec_lab.log 2>&1
echo DEC_OK
timeout -k 10 240 python3 tools/bs_lab.py run --reps 10 --out $OUT/bs_lab.json > $OUT/bs_lab.log 2>&1
echo ENC_OK
