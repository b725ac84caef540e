#!/bin/bash
# Round-2 evidence on one GPU box: the profile round (kernel stats, PMC
# traffic, SQ counters, full bench) then the C5 shapes incl. the mixed
# heterogeneous batch.  Any failing step stops the script.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=r02 bash tools/profile_round.sh
timeout -k 10 500 python3 tools/bench_c5.py --out gpurun_out/profiles/r02_c5_bench.json > gpurun_out/c5.log 2>&1
echo R02_OK
