#!/bin/bash
# GPU box, round 4: decode/encode GPU tests, the default bench line, then the
# kernel trace, SQ counters and FETCH / WRITE passes of the bench workload
# (profiles keyed on the built kernels' code hashes), and the native
# per-packet driver (tools/bench_on_send.cpp).   TAG=r04e tools/gpu_r04_prof.sh
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-r04}
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ "${WITH_TESTS:-1}" = "1" ]; then
  timeout -k 10 500 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_fullsize.py tests/test_gpu_encode.py \
      tests/test_gpu_abi_c.py -x -q --timeout 170 --timeout-method thread > $OUT/gpu_tests.log 2>&1
  tail -2 $OUT/gpu_tests.log
fi
timeout -k 10 400 python3 bench.py > $OUT/bench_full.log 2>&1
tail -1 $OUT/bench_full.log | cut -c1-300
ARGS="--steps 3 --warmup 1 --no-cpu --host-path-G 0 --c3b-G 0 --c4-G 0 --c5-mixed-bytes 0"
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
timeout -k 10 200 tools/send_batch/build/bench_on_send 300 > $OUT/on_send_native.json 2> $OUT/on_send_native.err
echo NATIVE_OK
