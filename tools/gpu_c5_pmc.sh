#!/bin/bash
# GPU box: SQ counters of the C5 (128, 20) block decode (synw + k_combine_slots).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/c5pmc
SH="${C5_SHAPES:-128,20}"
timeout -k 10 120 python3 tools/bench_c5.py --shapes "$SH" --modes block --reps 3 --bytes 2e9 \
    --out gpurun_out/c5pmc/plain.json > gpurun_out/c5pmc/plain.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5pmc/kt -o kt -- \
    python3 tools/bench_c5.py --shapes "$SH" --modes block --reps 3 --bytes 2e9 --out /tmp/x.json \
    > gpurun_out/c5pmc/kt.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT \
    SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/c5pmc/p1 -o p1 -- \
    python3 tools/bench_c5.py --shapes "$SH" --modes block --reps 1 --bytes 2e9 --out /tmp/x.json \
    > gpurun_out/c5pmc/p1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_LDS --output-format csv -d gpurun_out/c5pmc/p2 -o p2 -- \
    python3 tools/bench_c5.py --shapes "$SH" --modes block --reps 1 --bytes 2e9 --out /tmp/x.json \
    > gpurun_out/c5pmc/p2.log 2>&1
echo C5PMC_OK
