#!/bin/bash
# Step schedule sweep on the GPU box: the headline bench (no side legs) under
# alternating settings, N rounds each.   TAG=r05d tools/sched_sweep.sh
#   SWEEP="label:ENV=val:bench args;label2:..."  (default: acceptance-pass grid caps)
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-r05}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
BASE="--steps 20 --warmup 5 --no-cpu --host-path-G 0 --c3b-G 0 --c4-G 0 --c5-mixed-bytes 0 --detail /tmp/sweep_detail.json"
SWEEP=${SWEEP:-"cap256:QF_PREPARE_GRID=0:;cap64:QF_PREPARE_GRID=64:;cap128:QF_PREPARE_GRID=128:;cap512:QF_PREPARE_GRID=512:;serial:QF_PREPARE_GRID=0:--serial"}
ROUNDS=${ROUNDS:-2}
: > "$OUT/sweep.jsonl"
for rnd in $(seq 1 "$ROUNDS"); do
  IFS=';' read -ra ITEMS <<< "$SWEEP"
  for it in "${ITEMS[@]}"; do
    IFS=':' read -r label envset args <<< "$it"
    line=$(env $envset timeout -k 10 120 python3 bench.py $BASE $args 2>/dev/null | grep '^{"metric"')
    python3 - "$label" "$rnd" "$line" >> "$OUT/sweep.jsonl" <<'PY'
import json, sys
label, rnd, line = sys.argv[1], int(sys.argv[2]), sys.argv[3]
d = json.loads(line)
re_ = d.get("roofline_encode") or {}
print(json.dumps({"label": label, "round": rnd, "value": d["value"], "ms_per_step": d["ms_per_step"],
                  "kernels": d.get("kernel_ms_per_launch"), "enc_in_step": (re_.get("in_step") or {}).get("launch_ms"),
                  "enc_alone": re_.get("launch_ms")}))
PY
    tail -1 "$OUT/sweep.jsonl"
  done
done
