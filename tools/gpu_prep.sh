set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_decode.py tests/test_gpu_fullsize.py tests/test_gpu_desc.py > gpurun_out/prep_tests.log 2>&1
timeout -k 10 300 python bench.py --no-cpu --host-path-G 0 --c3b-G 0 > gpurun_out/prep_bench.log 2>&1
echo PREP_OK
