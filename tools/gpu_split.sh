#!/bin/bash
# GPU box: split-phase decode (acceptance pass beside the encode; the bench
# default) vs serial, twice each, alternating.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03}
mkdir -p $OUT
ARGS="--no-cpu --host-path-G 0 --c3b-G 0 --c4-G 0 --steps 20"
run() { local name=$1; shift; env "$@" timeout -k 10 200 python bench.py $ARGS $EXTRA > $OUT/sp_$name.log 2>&1; }
EXTRA="--serial" run serial
EXTRA="" run split
EXTRA="--serial" run serial2
EXTRA="" run split2
EXTRA="" run split_g512 QF_PREPARE_GRID=512
for f in serial split serial2 split2 split_g512; do python3 -c "
import json; d=json.loads(open('$OUT/sp_$f.log').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'], d.get('encode_ms'), d.get('decode_ms'), d['kernel_ms_per_launch'], d['verified'])"; done
