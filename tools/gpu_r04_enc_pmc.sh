#!/bin/bash
# GPU box, round 4: encode lab timing + FETCH_SIZE / WRITE_SIZE per lab kernel
# (cache policy of the row loads vs the 8 % read over-fetch).
#   TAG=r04a tools/gpu_r04_enc_pmc.sh      (after: python tools/bs_lab.py build)
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-r04a}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 240 python3 tools/bs_lab.py run --reps 10 --out $OUT/bs_lab.json > $OUT/bs_lab.log 2>&1
echo LAB_OK
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/lf -o run -- python3 tools/bs_lab.py run --reps 3 --out $OUT/bs_lab_f.json > $OUT/lf.log 2>&1
echo FETCH_OK
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/lw -o run -- python3 tools/bs_lab.py run --reps 3 --out $OUT/bs_lab_w.json > $OUT/lw.log 2>&1
echo WRITE_OK
python3 tools/lab_pmc.py $OUT/lf $OUT/lw --out $OUT/traffic_lab.json \
  --command "rocprofv3 --pmc FETCH_SIZE | --pmc WRITE_SIZE (separate runs) -- python3 tools/bs_lab.py run --reps 3"
