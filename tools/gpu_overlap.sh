#!/bin/bash
# GPU box: encode || decode on two streams with persistent-grid caps (QF_*_BLOCKS_PER_CU).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
out=gpurun_out/overlap.txt; : > $out
run() {   # run <extra bench args> <env assignments...>
  local extra="$1"; shift
  echo "== $extra $*" >> $out
  env "$@" timeout -k 10 200 python bench.py --no-cpu --host-path-G 0 --c3b-G 0 --steps 10 $extra > gpurun_out/ov.log 2>&1 || { echo FAIL >> $out; return 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/ov.log').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['encode_ms'], d['decode_ms'], d['verified'], d['kernel_ms_per_launch'])" >> $out
}
run "" QF_X=0 && \
run "--overlap" QF_X=0 && \
run "" QF_ENC_BLOCKS_PER_CU=1 QF_DEC_BLOCKS_PER_CU=1 && \
run "--overlap" QF_ENC_BLOCKS_PER_CU=1 QF_DEC_BLOCKS_PER_CU=1 && \
run "--overlap" QF_ENC_BLOCKS_PER_CU=2 QF_DEC_BLOCKS_PER_CU=1 && \
run "--overlap" QF_ENC_BLOCKS_PER_CU=1 QF_DEC_BLOCKS_PER_CU=2
cat $out
