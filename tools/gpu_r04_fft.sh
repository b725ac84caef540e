#!/bin/bash
# GPU box, round 4: GF(2^16) tests, the GF(2^16) bench (FFT variants) and the
# SQ counters of the FFT encode (16 Extreme windows).   TAG=r04i tools/gpu_r04_fft.sh
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-r04}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_gf16.py -x -q --timeout 170 --timeout-method thread > $OUT/gf16_tests.log 2>&1 || { tail -30 $OUT/gf16_tests.log; exit 1; }
tail -2 $OUT/gf16_tests.log
timeout -k 10 300 python tools/bench_gf16.py --out $OUT/gf16_bench.json > $OUT/gf16_bench.log 2>&1
tail -1 $OUT/gf16_bench.log
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS --output-format csv -d $OUT/pmc_fft16 -o run -- python3 tools/fft16_probe.py > $OUT/pmc_fft16.log 2>&1
python3 tools/sq_summary.py $OUT/pmc_fft16 $OUT/fft16_sq.json | grep -A12 fft16
