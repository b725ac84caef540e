set -e
O=gpurun_out/${TAG:-r05an}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 170 --timeout-method thread tests/test_gpu_decode.py tests/test_gpu_c5_mixed.py -k "${TESTK:-96 or 48 or c5 or mixed}" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
  timeout -k 10 200 python3 tools/bench_c5.py --shapes "${SHAPES:-96,15;48,8}" --modes block --reps 5 --out $O/a$i.json > $O/a$i.log 2>&1
  QF_FFT_KERNELS=0 timeout -k 10 200 python3 tools/bench_c5.py --shapes "${SHAPES:-96,15;48,8}" --modes block --reps 5 --out $O/b$i.json > $O/b$i.log 2>&1
done
for f in a1 b1 a2 b2; do echo "== $f"; grep "^k" $O/$f.log; done
