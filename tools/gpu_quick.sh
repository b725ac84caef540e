#!/bin/bash
# Quick GPU iteration: selected GPU tests (TESTS), then one bench run (BENCH_ARGS).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest ${TESTS:-tests} -m gpu -q -x --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_quick.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_quick.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench_quick.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/bench_quick.log; exit $rc
