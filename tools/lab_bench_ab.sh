# bench line A/B over environment variants (VARIANTS="name:ENV=val ..."), alternating twice;
# prints value / encode in-step frac / decode ms per run
set -e
O=gpurun_out/${TAG:-r05ab}; mkdir -p $O
ARGS="--steps 20 --warmup 5 --no-cpu --host-path-G 0 --c3b-G 0 --c4-G 0 --c5-mixed-bytes 0 --c5-shape-bytes 0"
for i in 1 2; do
  for v in $VARIANTS; do
    name=${v%%:*}; envs=${v#*:}; [ "$envs" = "$v" ] && envs=""
    env $envs timeout -k 10 300 python3 bench.py --detail "" $ARGS > $O/${name}_$i.log 2>&1
    python3 - "$O/${name}_$i.log" "$name" <<'PY'
import json, sys
line = next(l for l in open(sys.argv[1]) if l.startswith('{"metric"'))
d = json.loads(line)
print(sys.argv[2], d["value"], d["ms_per_step"], d["roofline_encode"]["in_step"], d["kernel_ms_per_launch"], flush=True)
PY
  done
done
