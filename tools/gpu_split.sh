#!/bin/bash
# Split-phase decode: bench serial vs --split at several acceptance-pass grid caps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider -k payload_wait > gpurun_out/pytest_split.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_split.log; [ $rc -eq 0 ] || exit $rc
for cfg in "0 " "64 --split" "128 --split" "256 --split" "512 --split" "1024 --split" "0 "; do
  set -- $cfg; export QF_PREPARE_GRID=$1; mode=${2:-}
  timeout -k 10 300 python bench.py --no-cpu --host-path-G 0 $mode > gpurun_out/bench_split.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "bench $cfg rc=$rc"; tail -5 gpurun_out/bench_split.log; exit $rc; }
  python - "$cfg" <<'PY'
import json, sys
d = json.loads([l for l in open("gpurun_out/bench_split.log") if l.startswith("{")][-1])
print(sys.argv[1], d["value"], d["ms_per_step"], d["encode_ms"], d["decode_ms"], d["kernel_ms_per_launch"], d["verified"])
PY
done
