#!/bin/bash
# GPU box, end of round 3: kernel trace, SQ counters and FETCH/WRITE passes of
# the default bench workload, the C5 shapes, the per-packet fec_modes and the
# GF(2^16) batched rates on the final tree.   TAG=r03 tools/gpu_r03_final.sh
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-r03}
OUT=gpurun_out/$TAG
mkdir -p $OUT
ARGS="--steps 3 --warmup 1 --no-cpu --host-path-G 0 --c3b-G 0 --c4-G 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 bench.py $ARGS > $OUT/kt.log 2>&1
grep '^{"metric"' $OUT/kt.log > $OUT/kt.bench.json
python3 tools/prof_summary.py $OUT/kt $OUT/kernel_stats.json --command "rocprofv3 --kernel-trace --stats --output-format csv -- python3 bench.py $ARGS"
echo KT_OK
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY --output-format csv -d $OUT/sq -o run -- python3 bench.py $ARGS > $OUT/sq.log 2>&1
python3 tools/sq_summary.py $OUT/sq $OUT/sq_counters.json > /dev/null
echo SQ_OK
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 bench.py $ARGS > $OUT/write.log 2>&1
python3 tools/pmc_traffic.py $OUT/fetch $OUT/write --k 64 --r 16 --L 1200 --G 65536 --out $OUT/traffic.json \
  --command "rocprofv3 --pmc FETCH_SIZE | --pmc WRITE_SIZE (separate runs) -- python3 bench.py $ARGS"
echo PMC_OK
timeout -k 10 400 python3 tools/bench_c5.py --out $OUT/c5_bench.json > $OUT/c5.log 2>&1
echo C5_OK
timeout -k 10 300 python3 tools/bench_fec_modes.py --out $OUT/fec_modes.json > $OUT/fec_modes.log 2>&1
echo MODES_OK
timeout -k 10 300 python3 tools/bench_gf16.py --out $OUT/gf16_bench.json > $OUT/gf16.log 2>&1
echo FINAL_OK
