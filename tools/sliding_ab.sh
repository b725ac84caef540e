set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-r06s}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -q --timeout 170 --timeout-method thread tests/test_gpu_encode.py -k "sliding" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for i in 1 2; do
  timeout -k 10 200 python3 tools/bench_c5.py --shapes "64,10;96,15;128,20;32,5" --modes sliding --reps 5 --bytes 1e9 --out $OUT/sl_a$i.json > $OUT/sl_a$i.log 2>&1
  QF_SLIDING_KERNELS=0 timeout -k 10 200 python3 tools/bench_c5.py --shapes "64,10;96,15;128,20;32,5" --modes sliding --reps 5 --bytes 1e9 --out $OUT/sl_b$i.json > $OUT/sl_b$i.log 2>&1
done
for f in a1 b1 a2 b2; do echo "== $f"; grep "^k" $OUT/sl_$f.log; done
