# Round 6: write-request counters of the fused grouping's
# kernels at 12.5 M and 100 M rows -- all L2->fabric write requests and the
# 64-byte ones (the rest are 32-byte, partial-line writes), then WRITE_SIZE --
# one rocprofv3 --pmc pass per set (no tracing in the same run); then the
# N = 2 / 3 bench rehearsal over the host transport with --verify.
#   TAG=r6g bash scripts/gpu_r6_wrreq.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/wrreq_$TAG
mkdir -p "$OUT"
SETS=("TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" "WRITE_SIZE" "TCC_EA0_WRREQ_DRAM_sum TCC_EA0_RDREQ_sum")
for rows in 12500000 100000000; do
  i=0
  for C in "${SETS[@]}"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $C -d "$OUT/r${rows}_s$i" -o pmc --output-format csv \
      -- python3 scripts/exp/exp_seg_groups.py $rows 2 > "$OUT/r${rows}_s$i.log" 2>&1 || exit 1
  done
done
python3 scripts/exp/pmc_kernels.py "$OUT" > "$OUT/summary.txt" || exit 1
cat "$OUT/summary.txt"
if [ -z "$NOVERIFY" ]; then
  for N in 2 3; do
    SD_BENCH_BACKEND=host timeout -k 10 400 python -u bench.py --gpus $N --steps 3 --warmup 1 \
      --components dedup --dedup-rows 4000000 --no-cpu --verify \
      > "$OUT/verify_host$N.json" 2> "$OUT/verify_host$N.err" || exit 1
    grep "verify:" "$OUT/verify_host$N.err"
  done
fi
