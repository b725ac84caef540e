#!/bin/bash
# The one GPU-box launcher (replaces the per-round tools/gpu_r0*_*.sh; those
# are in git history before round 5).  Every GPU step has its own time limit
# and any failure ends the script (set -e, steps chained).
#
#   TAG=r05a tools/gpu.sh tests [pytest args...]   -m gpu suite (or the files given)
#   TAG=r05a tools/gpu.sh full                     -m gpu suite, smoke, one default bench line
#   TAG=r05a tools/gpu.sh bench [bench args...]    one bench line (+ detail record)
#   TAG=r05a tools/gpu.sh prof                     bench line, kernel trace, SQ counters, FETCH / WRITE passes
#   TAG=r06a tools/gpu.sh cmblab                   payload-pass lab (tools/cmb_lab.py) + FETCH / WRITE per variant
#   TAG=r05a tools/gpu.sh run <command...>         any command, under a 600 s limit
#   TAG=r05a C5_SHAPES="196,59;160,48" AB_ENV=QF_SYNW_SHARED=0 [C5_TESTK="..."] tools/gpu.sh c5ab
#        C5 GPU tests, then block GiB/s of the shapes: library (a) against AB_ENV (b), alternating twice
#   TAG=r05a VARIANTS="lib g128:QF_PREPARE_GRID=128" tools/gpu.sh benchab
#        the headline step under environment variants, alternating twice (value, encode in-step, kernel ms)
#
# Outputs: gpurun_out/$TAG/ (merged back by gpurun; copy what is judged into profiles/).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-r05}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
what=${1:-full}
shift || true
PYT="python -u -m pytest -x -q --timeout 170 --timeout-method thread"
ARGS="--steps 20 --warmup 5 --no-cpu --host-path-G 0 --c3b-G 0 --c4-G 0 --c5-mixed-bytes 0"

bench_line() {   # $1 log name, rest: bench args
  local name=$1
  shift
  timeout -k 10 400 python3 bench.py --detail "$OUT/${name}_detail.json" "$@" > "$OUT/$name.log" 2>&1
  grep '^{"metric"' "$OUT/$name.log" > "$OUT/$name.json"
  echo "$name: $(wc -c < "$OUT/$name.json") bytes"
  cut -c1-300 "$OUT/$name.json"
}

case "$what" in
  tests)
    if [ $# -eq 0 ]; then set -- tests -m gpu; fi
    timeout -k 10 1000 $PYT "$@" > "$OUT/gpu_tests.log" 2>&1 || { tail -30 "$OUT/gpu_tests.log"; exit 1; }
    tail -3 "$OUT/gpu_tests.log"
    ;;
  full)
    timeout -k 10 1000 $PYT tests -m gpu > "$OUT/gpu_tests.log" 2>&1 || { tail -30 "$OUT/gpu_tests.log"; exit 1; }
    tail -3 "$OUT/gpu_tests.log"
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > "$OUT/smoke.log" 2>&1
    tail -1 "$OUT/smoke.log"
    bench_line bench_full
    ;;
  bench)
    bench_line bench_full "$@"
    ;;
  prof)
    bench_line bench_full
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- \
      python3 bench.py --detail "$OUT/kt_detail.json" $ARGS > "$OUT/kt.log" 2>&1
    grep '^{"metric"' "$OUT/kt.log" > "$OUT/kt.bench.json"
    python3 tools/prof_summary.py "$OUT/kt" "$OUT/kernel_stats.json" \
      --command "rocprofv3 --kernel-trace --stats --output-format csv -- python3 bench.py $ARGS"
    echo KT_OK
    timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_LDS \
      SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY --output-format csv -d "$OUT/sq" -o run -- \
      python3 bench.py --detail "" $ARGS > "$OUT/sq.log" 2>&1
    python3 tools/sq_summary.py "$OUT/sq" "$OUT/sq_counters.json" > /dev/null
    echo SQ_OK
    timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- \
      python3 bench.py --detail "" $ARGS > "$OUT/fetch.log" 2>&1
    timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- \
      python3 bench.py --detail "" $ARGS > "$OUT/write.log" 2>&1
    python3 tools/pmc_traffic.py "$OUT/fetch" "$OUT/write" --k 64 --r 16 --L 1200 --G 65536 --out "$OUT/traffic.json" \
      --command "rocprofv3 --pmc FETCH_SIZE | --pmc WRITE_SIZE (separate runs) -- python3 bench.py $ARGS"
    echo PMC_OK
    ;;
  schedab)  # the headline step, default (split) schedule against --overlap, twice each
    for i in 1 2; do
      for m in split overlap; do
        X=""; [ "$m" = overlap ] && X="--overlap"
        timeout -k 10 200 python3 bench.py --no-cpu --c3b-G 0 --host-path-G 0 --c5-mixed-bytes 0 --steps 20 \
          --warmup 5 --detail "" $X > "$OUT/$m$i.log" 2>&1
      done
    done
    for f in split1 overlap1 split2 overlap2; do echo "== $f"; grep '^{"metric"' "$OUT/$f.log" | cut -c1-200; done
    ;;
  declab)   # tools/dec_lab.py run (build the variants here first: python tools/dec_lab.py build)
    timeout -k 10 300 python3 tools/dec_lab.py run --reps 10 --out "$OUT/dec_lab.json" "$@" > "$OUT/dec_lab.log" 2>&1
    tail -20 "$OUT/dec_lab.log"
    ;;
  cmblab)   # tools/cmb_lab.py run + FETCH / WRITE passes per variant (build here first: python tools/cmb_lab.py build)
    CL="python3 tools/cmb_lab.py run --reps 10"
    timeout -k 10 300 $CL --out "$OUT/cmb_lab.json" > "$OUT/cmb_lab.log" 2>&1
    tail -12 "$OUT/cmb_lab.log"
    timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/cmbfetch" -o f -- \
      $CL --reps 2 --out /tmp/cmbx.json > "$OUT/cmbfetch.log" 2>&1
    timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/cmbwrite" -o w -- \
      $CL --reps 2 --out /tmp/cmbx.json > "$OUT/cmbwrite.log" 2>&1
    python3 tools/c5_pmc_summary.py "$OUT/cmbfetch" "$OUT/cmbwrite" --match cmb_ --out "$OUT/cmb_pmc.json"
    echo CMBLAB_OK
    ;;
  c5pmc)    # counters of the C5 kernels of one shape (C5_SHAPES, default 196,59): block encode + decode
    SH="${C5_SHAPES:-196,59}"
    BC="python3 tools/bench_c5.py --shapes $SH --modes block --reps 3 --bytes 2e9"
    timeout -k 10 200 $BC --out "$OUT/c5_plain.json" > "$OUT/c5_plain.log" 2>&1
    tail -2 "$OUT/c5_plain.log"
    timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c5kt" -o kt -- \
      $BC --out /tmp/c5x.json > "$OUT/c5kt.log" 2>&1
    timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES \
      SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_ANY --output-format csv -d "$OUT/c5sq" -o sq -- \
      $BC --out /tmp/c5x.json > "$OUT/c5sq.log" 2>&1
    timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/c5fetch" -o f -- \
      $BC --out /tmp/c5x.json > "$OUT/c5fetch.log" 2>&1
    timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/c5write" -o w -- \
      $BC --out /tmp/c5x.json > "$OUT/c5write.log" 2>&1
    python3 tools/c5_pmc_summary.py "$OUT/c5sq" "$OUT/c5fetch" "$OUT/c5write" --out "$OUT/c5_pmc.json"
    python3 tools/prof_summary.py "$OUT/c5kt" "$OUT/c5_kernel_stats.json" --command "rocprofv3 --kernel-trace --stats -- $BC"
    echo C5PMC_OK
    ;;
  c5sq)     # SQ counters of the C5 sliding-window encodes, all seven shapes -> profiles/c5_sq_counters.json
    SH="32,5;48,8;64,10;96,15;128,20;160,48;196,59"
    BC="python3 tools/bench_c5.py --shapes $SH --modes sliding --reps 3 --bytes 1e9"
    timeout -k 10 300 $BC --out "$OUT/c5sl_plain.json" > "$OUT/c5sl_plain.log" 2>&1
    grep "^k" "$OUT/c5sl_plain.log"
    timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
      SQ_WAIT_INST_ANY SQ_INSTS_LDS --output-format csv -d "$OUT/c5slsq" -o sq -- \
      $BC --out "$OUT/c5sl_sq.json" > "$OUT/c5slsq.log" 2>&1
    cp profiles/c5_sq_counters.json "$OUT/c5_sq_counters.json" 2>/dev/null || true
    python3 tools/c5_sq_summary.py "$OUT/c5slsq" "$OUT/c5sl_sq.json" --mode sliding --out "$OUT/c5_sq_counters.json" \
      --command "rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS -- $BC"
    echo C5SQ_OK
    ;;
  c5ab)
    SH="${C5_SHAPES:-196,59;160,48;128,39}"
    TK="${C5_TESTK:-c5 or passes or merged or 196 or synw or large or 96 or 48}"
    timeout -k 10 600 $PYT tests/test_gpu_c5_mixed.py tests/test_gpu_encode.py tests/test_gpu_decode.py -k "$TK" \
      > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
    tail -2 "$OUT/tests.log"
    for i in 1 2; do
      timeout -k 10 200 python3 tools/bench_c5.py --shapes "$SH" --modes block --reps 5 --out "$OUT/c5_a$i.json" \
        > "$OUT/c5_a$i.log" 2>&1
      env ${AB_ENV:-QF_SYNW_SHARED=0} timeout -k 10 200 python3 tools/bench_c5.py --shapes "$SH" --modes block \
        --reps 5 --out "$OUT/c5_b$i.json" > "$OUT/c5_b$i.log" 2>&1
    done
    for f in a1 b1 a2 b2; do echo "== $f"; grep "^k" "$OUT/c5_$f.log"; done
    ;;
  benchab)
    AB_ARGS="$ARGS --c5-shape-bytes 0"
    for i in 1 2; do
      for v in ${VARIANTS:-lib}; do
        name=${v%%:*}; envs=${v#*:}; [ "$envs" = "$v" ] && envs=""
        env $envs timeout -k 10 300 python3 bench.py --detail "" $AB_ARGS > "$OUT/${name}_$i.log" 2>&1
        python3 - "$OUT/${name}_$i.log" "$name" <<'PY'
import json, sys
d = json.loads(next(l for l in open(sys.argv[1]) if l.startswith('{"metric"')))
print(sys.argv[2], d["value"], d["ms_per_step"], d["roofline_encode"]["in_step"], d["kernel_ms_per_launch"], flush=True)
PY
      done
    done
    ;;
  run)
    timeout -k 10 600 "$@"
    ;;
  *)
    echo "unknown: $what" >&2
    exit 2
    ;;
esac
