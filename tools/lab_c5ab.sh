# C5 check after a library change: the C5 GPU tests, then block GiB/s of the
# large shapes with an option on / off (AB_ENV="QF_X=0"), alternating twice
set -e
O=gpurun_out/${TAG:-r05v}; mkdir -p $O
SH=${C5_SHAPES:-"196,59;160,48;128,39"}
timeout -k 10 600 python -u -m pytest -x -q --timeout 170 --timeout-method thread tests/test_gpu_c5_mixed.py tests/test_gpu_encode.py tests/test_gpu_decode.py -k "c5 or passes or merged or 196 or synw or large" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
  timeout -k 10 200 python3 tools/bench_c5.py --shapes "$SH" --modes block --reps 5 --out $O/c5_a$i.json > $O/c5_a$i.log 2>&1
  env ${AB_ENV:-QF_SYNW_SHARED=0} timeout -k 10 200 python3 tools/bench_c5.py --shapes "$SH" --modes block --reps 5 --out $O/c5_b$i.json > $O/c5_b$i.log 2>&1
done
for f in a1 b1 a2 b2; do echo "== $f"; grep "^k" $O/c5_$f.log; done
