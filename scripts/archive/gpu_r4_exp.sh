# Round-4 kernel experiment: run build/$EXP with args, then (PROF=1) its
# rocprofv3 kernel trace and FETCH_SIZE / WRITE_SIZE passes, separately.
#   TAG=r4x EXP=exp_repwrite bash scripts/gpu_r4_exp.sh 100000000 10
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG}_${EXP}
mkdir -p "$OUT"
timeout -k 10 240 build/$EXP "$@" > "$OUT/run_$1.log" 2>&1 || { cat "$OUT/run_$1.log"; exit 1; }
cat "$OUT/run_$1.log"
if [ -n "$PROF" ]; then
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/trace_$1" -o run --output-format csv \
    -- build/$EXP "$@" > "$OUT/trace_$1.log" 2>&1 || exit 1
  python3 scripts/trace_summary.py "$OUT/trace_$1/run_kernel_trace.csv" "$OUT/trace_summary_$1.txt" > /dev/null || exit 1
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $C -d "$OUT/pmc_$1/pmc_$C" -o pmc --output-format csv \
      -- build/$EXP "$@" > "$OUT/pmc_${1}_$C.log" 2>&1 || exit 1
  done
  python3 scripts/pmc_summary.py "$OUT/pmc_$1" "$OUT/pmc_$1.json" > "$OUT/pmc_$1.txt" || exit 1
  cat "$OUT/pmc_$1.txt"
fi
