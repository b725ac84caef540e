cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python tools/bs_lab.py run --reps 20 > gpurun_out/lab.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_encode.py tests/test_gpu_decode.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_gpu.log; cat gpurun_out/lab.log | grep -v amdgpu.ids
[ $rc -eq 0 ] && timeout -k 10 300 python bench.py --no-cpu --host-path-G 0 > gpurun_out/bench.log 2>&1; tail -2 gpurun_out/bench.log
