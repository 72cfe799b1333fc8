#!/bin/bash
# rocprofv3 captures for profiles/ (run on the GPU box via gpurun):
#   1) kernel trace + stats of a short bench run (per-kernel average durations)
#   2) separate PMC passes (never combined with tracing domains): HBM bytes
#      (FETCH_SIZE / WRITE_SIZE, one per pass) and SQ VALU counters.
# Usage: TAG=r1 bash scripts/profile.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${TAG:-r1}
OUT=gpurun_out/prof_$T
mkdir -p "$OUT"
ARGS="--steps 3 --warmup 1 --no-cpu ${BENCH_ARGS:-}"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
  -- python3 bench.py $ARGS > "$OUT/trace_bench.json" 2> "$OUT/trace_bench.err" || exit $?
python3 scripts/trace_summary.py "$OUT/trace/run_kernel_trace.csv" "$OUT/trace_summary.txt" > /dev/null || exit 1
if [ -n "$PMC" ]; then
  rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
  PARGS="--steps 1 --warmup 0 --no-cpu ${PMC_ARGS:---components cas}"
  for C in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
    N=$(echo $C | tr ' ' '_')
    timeout -s KILL 240 rocprofv3 --pmc $C -d "$OUT/pmc_$N" -o pmc --output-format csv \
      -- python3 bench.py $PARGS > "$OUT/pmc_$N.log" 2>&1 || { echo "pmc $C failed: $?"; exit 1; }
  done
  python3 scripts/pmc_summary.py "$OUT" "$OUT/pmc_traffic.json" > "$OUT/pmc_traffic.txt" || exit 1
fi
echo done
