#!/bin/bash
# GPU box, round 4: HBM fetch and SQ counters of the C5 pass kernels (merged
# dispatch, default options) at 1 GB of source per shape.   TAG=r04w tools/gpu_r04_c5traffic.sh
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-r04}
OUT=gpurun_out/$TAG
mkdir -p $OUT
SH="${C5_SHAPES:-128,39;160,48;196,59}"
ARGS="--shapes $SH --modes block --reps 1 --bytes 1e9"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- \
    python3 tools/bench_c5.py $ARGS --out $OUT/f.json > $OUT/fetch.log 2>&1
echo FETCH_OK
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY \
    SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_WAIT_ANY --output-format csv -d $OUT/sq -o run -- \
    python3 tools/bench_c5.py $ARGS --out $OUT/s.json > $OUT/sq.log 2>&1
echo SQ_OK
python3 tools/c5_pmc_summary.py $OUT/fetch $OUT/sq --out $OUT/c5_pmc.json
