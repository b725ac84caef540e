#!/bin/bash
# rocprofv3 evidence for the bench workload (run on the GPU box):
#   1. --kernel-trace --stats        -> gpurun_out/profiles/${TAG}_kernel_stats.json (+ .bench.json of that run)
#   2. --pmc FETCH_SIZE (own pass)   \
#   3. --pmc WRITE_SIZE (own pass)   -> profiles/traffic.json
#   4. --pmc SQ_* (own pass)         -> gpurun_out/profiles/${TAG}_sq_counters.json
#   5. plain bench (CPU baseline on) -> gpurun_out/profiles/${TAG}_bench_full.json
# Outputs go to gpurun_out/profiles/ (merged back by gpurun; copy into profiles/).
# Every GPU step has its own time limit; any failure stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r01}
ARGS="--steps 3 --warmup 1 --no-cpu --host-path-G 0"
set -e
mkdir -p gpurun_out/profiles
rm -rf gpurun_out/prof gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/pmc_sq
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py $ARGS > gpurun_out/prof_bench.log 2>&1
grep "^{\"metric\"" gpurun_out/prof_bench.log > gpurun_out/profiles/${TAG}_kernel_stats.bench.json
python3 tools/prof_summary.py gpurun_out/prof gpurun_out/profiles/${TAG}_kernel_stats.json \
  --command "rocprofv3 --kernel-trace --stats --output-format csv -- python3 bench.py $ARGS"
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 bench.py $ARGS > gpurun_out/pmc_fetch.log 2>&1
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python3 bench.py $ARGS > gpurun_out/pmc_write.log 2>&1
python3 tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write --k 64 --r 16 --L 1200 --G 65536 --out gpurun_out/profiles/traffic.json \
  --command "rocprofv3 --pmc FETCH_SIZE | --pmc WRITE_SIZE (separate runs) -- python3 bench.py $ARGS"
timeout -s KILL 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY --output-format csv -d gpurun_out/pmc_sq -o run -- python3 bench.py $ARGS > gpurun_out/pmc_sq.log 2>&1
python3 tools/sq_summary.py gpurun_out/pmc_sq gpurun_out/profiles/${TAG}_sq_counters.json > /dev/null
cp gpurun_out/profiles/traffic.json profiles/traffic.json   # the bench line reads it (traffic field)
timeout -k 10 400 python3 bench.py > gpurun_out/bench_full.log 2>&1
grep "^{\"metric\"" gpurun_out/bench_full.log > gpurun_out/profiles/${TAG}_bench_full.json
echo PROFILE_OK
