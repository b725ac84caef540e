#!/bin/bash
# GPU box, round 4b: pool-block (1,280-B) row strides against dense rows, encode
# and fused decode labs, timing + FETCH/WRITE per lab kernel.
#   TAG=r04b tools/gpu_r04_layout.sh   (after: python tools/bs_lab.py build && python tools/dec_lab.py build)
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-r04b}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 240 python3 tools/bs_lab.py run --reps 10 --out $OUT/bs_lab.json > $OUT/bs_lab.log 2>&1
echo ENC_OK
timeout -k 10 240 python3 tools/dec_lab.py run --reps 10 --out $OUT/dec_lab.json > $OUT/dec_lab.log 2>&1
echo DEC_OK
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/lf -o run -- python3 tools/bs_lab.py run --reps 2 --out $OUT/x1.json > $OUT/lf.log 2>&1
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/lw -o run -- python3 tools/bs_lab.py run --reps 2 --out $OUT/x2.json > $OUT/lw.log 2>&1
python3 tools/lab_pmc.py $OUT/lf $OUT/lw --out $OUT/traffic_enc.json --command "rocprofv3 --pmc FETCH_SIZE | --pmc WRITE_SIZE -- python3 tools/bs_lab.py run --reps 2" > /dev/null
echo ENC_PMC_OK
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/df -o run -- python3 tools/dec_lab.py run --reps 2 --out $OUT/x3.json > $OUT/df.log 2>&1
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/dw -o run -- python3 tools/dec_lab.py run --reps 2 --out $OUT/x4.json > $OUT/dw.log 2>&1
python3 tools/lab_pmc.py $OUT/df $OUT/dw --dec --out $OUT/traffic_dec.json --command "rocprofv3 --pmc FETCH_SIZE | --pmc WRITE_SIZE -- python3 tools/dec_lab.py run --reps 2" > /dev/null
echo DEC_PMC_OK
