#!/bin/bash
# rocprofv3 evidence for the bench workload (run on the GPU box):
#   1. --kernel-trace --stats        -> profiles/${TAG}_kernel_stats.json
#   2. --pmc FETCH_SIZE (own pass)   \
#   3. --pmc WRITE_SIZE (own pass)   -> profiles/traffic.json
# Every GPU step has its own time limit; any failure stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r01}
ARGS="--steps 3 --warmup 1 --no-cpu --host-path-G 0"
set -e
rm -rf gpurun_out/prof gpurun_out/pmc_fetch gpurun_out/pmc_write
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py $ARGS > gpurun_out/prof_bench.log 2>&1
python3 tools/prof_summary.py gpurun_out/prof profiles/${TAG}_kernel_stats.json \
  --command "rocprofv3 --kernel-trace --stats --output-format csv -- python3 bench.py $ARGS"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 bench.py $ARGS > gpurun_out/pmc_fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python3 bench.py $ARGS > gpurun_out/pmc_write.log 2>&1
python3 tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write --k 64 --r 16 --L 1200 --G 65536 \
  --command "rocprofv3 --pmc FETCH_SIZE | --pmc WRITE_SIZE (separate runs) -- python3 bench.py $ARGS"
echo PROFILE_OK
