set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r04t
for B in 1e9 1.329e9 0.886e9 2.658e9; do
  for F in 0 1; do
    QF_FFT_KERNELS=$F timeout -k 10 120 python3 tools/bench_c5.py --shapes "160,48" --modes block --reps 5 --bytes $B --out gpurun_out/r04t/t_${B}_$F.json > gpurun_out/r04t/t_${B}_$F.log 2>&1
    echo "B=$B fft=$F $(grep k160 gpurun_out/r04t/t_${B}_$F.log)"
  done
done
