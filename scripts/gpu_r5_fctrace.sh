# Round 5: kernel timeline of the identifier job step through a one-rank RCCL
# communicator (SD_BENCH_FORCE_COMM=1) next to the fused one-GPU step.
#   TAG=r5g bash scripts/gpu_r5_fctrace.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/fctrace_$TAG
mkdir -p "$OUT"
for fc in 1 0; do
  SD_BENCH_FORCE_COMM=$fc timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/fc$fc" -o run \
    --output-format csv -- python3 bench.py --gpus 1 --steps 6 --warmup 2 --components cas \
    --no-cpu > "$OUT/fc$fc.json" 2> "$OUT/fc$fc.err" || exit 1
  f=$(find "$OUT/fc$fc" -name "run_kernel_trace.csv" | head -1)
  python3 scripts/exp/timeline.py "$f" ${TL_N:-60} > "$OUT/fc${fc}_timeline.txt" || exit 1
  echo "== fc$fc"; tail -22 "$OUT/fc${fc}_timeline.txt"
done
