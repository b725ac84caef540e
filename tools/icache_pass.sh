cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/icache
timeout -s KILL 60 rocprofv3 -L > gpurun_out/icache/avail.txt 2>&1 || true
grep -o "SQC_ICACHE[A-Z_]*" gpurun_out/icache/avail.txt | sort -u > gpurun_out/icache/names.txt
cat gpurun_out/icache/names.txt
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_MISSES SQC_ICACHE_HITS --output-format csv -d gpurun_out/icache/serial -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --host-path-G 0 > gpurun_out/icache/serial.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_MISSES SQC_ICACHE_HITS --output-format csv -d gpurun_out/icache/overlap -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --host-path-G 0 --overlap > gpurun_out/icache/overlap.log 2>&1
