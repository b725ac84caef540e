#!/bin/bash
# GPU box: SQ counters of the GF(2^16) FFT kernel (one --pmc pass, 8 SQ counters)
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-r03}
mkdir -p gpurun_out/profiles
rm -rf gpurun_out/pmc_fft16
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS --output-format csv -d gpurun_out/pmc_fft16 -o run -- python3 tools/fft16_probe.py > gpurun_out/pmc_fft16.log 2>&1
python3 tools/sq_summary.py gpurun_out/pmc_fft16 gpurun_out/profiles/${TAG}_fft16_sq.json | grep -A12 fft16
