# Kernel trace (rocprofv3 --kernel-trace --stats) of the dedup leg alone:
# per-kernel durations of the 12.5 M- and 100 M-row grouping / fused calls.
#   TAG=r4zd bash scripts/gpu_r4_dedup_trace.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
  -- python3 bench.py --steps 10 --warmup 2 --no-cpu --components dedup --no-exchange-model \
  --no-explicit-rank > "$OUT/trace_bench.json" 2> "$OUT/trace_bench.err" || exit 1
python3 scripts/trace_summary.py "$OUT/trace/run_kernel_trace.csv" "$OUT/trace_summary.txt" > /dev/null || exit 1
grep -E "k_list_finish|k_extra|k_part_private|k_part_hist|k_bucket_group12" "$OUT/trace_summary.txt" | head -30
