#!/bin/bash
# GPU box: bench step with persistent (capped) grids vs one item per wave.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03}
mkdir -p $OUT
ARGS="--no-cpu --host-path-G 0 --c3b-G 0 --c4-G 0 --steps 20"
timeout -k 10 200 python bench.py $ARGS > $OUT/cap_default.log 2>&1
QF_DEC_BLOCKS_PER_CU=2 timeout -k 10 200 python bench.py $ARGS > $OUT/cap_dec2.log 2>&1
QF_DEC_BLOCKS_PER_CU=2 QF_ENC_BLOCKS_PER_CU=2 timeout -k 10 200 python bench.py $ARGS > $OUT/cap_both2.log 2>&1
QF_ENC_BLOCKS_PER_CU=2 timeout -k 10 200 python bench.py $ARGS > $OUT/cap_enc2.log 2>&1
timeout -k 10 200 python bench.py $ARGS > $OUT/cap_default2.log 2>&1
for f in cap_default cap_dec2 cap_both2 cap_enc2 cap_default2; do python3 -c "
import json,sys; d=json.loads(open('$OUT/$f.log').read().strip().splitlines()[-1]); print('$f', d['value'], d['kernel_ms_per_launch'])"; done
