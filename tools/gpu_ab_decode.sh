#!/bin/bash
# A/B of the fused decode layouts on one box: decode GPU tests, then the bench
# with the chunked kernel (default) and the legacy one (QF_DECODE_LEGACY=1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_decode.py tests/test_gpu_fullsize.py tests/test_gpu_abi_c.py tests/test_gpu_desc.py} -m gpu -q -x --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ab.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_ab.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1 0 1; do
  QF_DECODE_LEGACY=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu --host-path-G 0 > gpurun_out/bench_ab_$v.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "bench rc=$rc"; exit $rc; }
  python - "$v" <<'PY'
import json,sys
d=json.loads([l for l in open(f"gpurun_out/bench_ab_{sys.argv[1]}.log") if l.startswith('{"metric"')][0])
print("legacy" if sys.argv[1]=="1" else "chunked", d["value"], d["ms_per_step"], d["kernel_ms_per_launch"])
PY
done
