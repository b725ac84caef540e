# C5 check after a library change: the C5 GPU tests, then block/sliding GiB/s of every shape
set -e
O=gpurun_out/${TAG:-r05v}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 170 --timeout-method thread tests/test_gpu_c5_mixed.py tests/test_gpu_encode.py tests/test_gpu_decode.py -k "c5 or passes or merged or 196 or synw or large" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python3 tools/bench_c5.py --reps 5 --out $O/c5.json > $O/c5.log 2>&1
tail -12 $O/c5.log
