# Round 5: timing + kernel timelines of the exchange path on one GPU
# (scripts/exp/exp_exchange_loop.py), one rocprofv3 trace per mode.
#   TAG=r5d bash scripts/gpu_r5_xtrace.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/xtrace_$TAG
mkdir -p "$OUT"
timeout -k 10 300 python3 scripts/exp/exp_exchange_loop.py > "$OUT/loop.json" 2> "$OUT/loop.err" || exit 1
cat "$OUT/loop.json"
for m in ${TRACE_MODES:-write_set_padded write_set_counted fused}; do
  MODES=$m timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/$m" -o run --output-format csv \
    -- python3 scripts/exp/exp_exchange_loop.py 12500000 8 > "$OUT/$m.json" 2> "$OUT/$m.err" || exit 1
  f=$(find "$OUT/$m" -name "run_kernel_trace.csv" | head -1)
  python3 scripts/exp/timeline.py "$f" ${TL_N:-40} > "$OUT/${m}_timeline.txt" || exit 1
  echo "== $m"; tail -14 "$OUT/${m}_timeline.txt"
done
