#!/bin/bash
# One GPU session: gpu tests -> smoke -> bench -> rocprofv3 kernel stats.
# Each GPU step has its own time limit; a fault/abort/timeout stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
stop() { echo "STOP after $1 rc=$2"; exit "$2"; }
ok_or_testfail() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }

timeout -k 10 900 python -m pytest tests -m gpu -q --timeout 300 -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
ok_or_testfail $rc || stop pytest $rc

timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
ok_or_testfail $rc || stop smoke $rc

timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench.log
ok_or_testfail $rc || stop bench $rc

if [ -n "${PROFILE:-}" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python bench.py --steps 5 --warmup 1 --no-cpu --host-path-G 0 > gpurun_out/prof.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -3 gpurun_out/prof.log
fi
exit 0
