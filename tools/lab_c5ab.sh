set -e
O=gpurun_out/r05t; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 170 --timeout-method thread tests/test_gpu_c5_mixed.py tests/test_gpu_encode.py tests/test_gpu_decode.py -k "c5 or passes or merged or 196 or synw" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
  timeout -k 10 200 python3 tools/bench_c5.py --shapes "196,59;160,48" --modes block --reps 5 --out $O/c5_fft$i.json > $O/c5_fft$i.log 2>&1
  QF_FFT_KERNELS=0 timeout -k 10 200 python3 tools/bench_c5.py --shapes "196,59;160,48" --modes block --reps 5 --out $O/c5_nofft$i.json > $O/c5_nofft$i.log 2>&1
done
tail -4 $O/c5_fft1.log $O/c5_nofft1.log $O/c5_fft2.log $O/c5_nofft2.log
