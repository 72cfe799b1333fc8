# Round-3 kernel experiments on one GPU box: run an experiment binary, then
# its rocprofv3 kernel trace and FETCH_SIZE / WRITE_SIZE passes (separately).
# Usage: TAG=r3x EXP=exp_xcd_scatter bash scripts/gpu_r3_exp.sh [args]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG}_${EXP}
mkdir -p "$OUT"
timeout -k 10 120 build/$EXP "$@" > "$OUT/run.log" 2>&1 || { cat "$OUT/run.log"; exit 1; }
cat "$OUT/run.log"
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
  -- build/$EXP "$@" > "$OUT/trace.log" 2>&1 || exit 1
python3 scripts/trace_summary.py "$OUT/trace/run_kernel_trace.csv" "$OUT/trace_summary.txt" > /dev/null || exit 1
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C -d "$OUT/pmc/pmc_$C" -o pmc --output-format csv \
    -- build/$EXP "$@" > "$OUT/pmc_$C.log" 2>&1 || exit 1
done
python3 scripts/pmc_summary.py "$OUT/pmc" "$OUT/pmc.json" > "$OUT/pmc.txt" || exit 1
cat "$OUT/pmc.txt"
