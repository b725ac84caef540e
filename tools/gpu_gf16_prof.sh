#!/bin/bash
# GPU box: rocprofv3 kernel trace of tools/bench_gf16.py (GF(2^16): bit-sliced,
# FFT and matvec kernels) -> gpurun_out/profiles/${TAG}_gf16_kernel_stats.json
#   TAG=r03am tools/gpu_gf16_prof.sh
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-r03}
mkdir -p gpurun_out/profiles
rm -rf gpurun_out/prof16
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof16 -o run -- python3 tools/bench_gf16.py --reps 3 --out gpurun_out/profiles/${TAG}_gf16_bench_under_prof.json > gpurun_out/prof16.log 2>&1
python3 tools/prof_summary.py gpurun_out/prof16 gpurun_out/profiles/${TAG}_gf16_kernel_stats.json \
  --command "rocprofv3 --kernel-trace --stats --output-format csv -- python3 tools/bench_gf16.py --reps 3"
echo PROF16_OK
