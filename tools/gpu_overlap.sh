#!/bin/bash
# GPU box: encode || decode on two streams (bench --overlap), with and without grid caps.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03}
mkdir -p $OUT
ARGS="--no-cpu --host-path-G 0 --c3b-G 0 --c4-G 0 --steps 20"
run() { local name=$1; shift; env "$@" timeout -k 10 200 python bench.py $ARGS $EXTRA > $OUT/ov_$name.log 2>&1; }
EXTRA="" run serial
EXTRA="--overlap" run ov
EXTRA="--overlap" run ov_e1d1 QF_ENC_BLOCKS_PER_CU=1 QF_DEC_BLOCKS_PER_CU=1
EXTRA="--overlap" run ov_e1 QF_ENC_BLOCKS_PER_CU=1
EXTRA="--overlap" run ov_d1 QF_DEC_BLOCKS_PER_CU=1
EXTRA="" run serial2
for f in serial ov ov_e1d1 ov_e1 ov_d1 serial2; do python3 -c "
import json; d=json.loads(open('$OUT/ov_$f.log').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'], d.get('encode_ms'), d.get('decode_ms'), d['kernel_ms_per_launch'])"; done
