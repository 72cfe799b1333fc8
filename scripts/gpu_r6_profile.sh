# Round-6 rocprofv3 captures (final tree): kernel trace + stats of a short bench run, then
# separate PMC passes (never combined with tracing): FETCH_SIZE / WRITE_SIZE /
# SQ VALU / GRBM over the config-2 K1 step, FETCH_SIZE / WRITE_SIZE over the
# 12.5 M-row grouping and over the 100 M-row (two-level) grouping; then the
# 2-rank rehearsal through bench --gpus 2 over libsdgpu's host transport (--verify).
# Usage: TAG=r6x bash scripts/gpu_r6_profile.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
  -- python3 bench.py --steps 3 --warmup 1 --no-cpu --staged-total-files 5000000 \
  > "$OUT/trace_bench.json" 2> "$OUT/trace_bench.err" || exit 1
python3 scripts/trace_summary.py "$OUT/trace/run_kernel_trace.csv" "$OUT/trace_summary.txt" > /dev/null || exit 1
for C in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  N=$(echo $C | tr ' ' '_')
  timeout -s KILL 240 rocprofv3 --pmc $C -d "$OUT/cas/pmc_$N" -o pmc --output-format csv \
    -- python3 bench.py --steps 1 --warmup 0 --no-cpu --components cas > "$OUT/cas_pmc_$N.log" 2>&1 || exit 1
done
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $C -d "$OUT/dedup/pmc_$C" -o pmc --output-format csv \
    -- python3 bench.py --steps 2 --warmup 1 --no-cpu --components dedup --dedup-full-rows 0 --no-explicit-rank --no-exchange-model \
    > "$OUT/dedup_pmc_$C.log" 2>&1 || exit 1
done
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $C -d "$OUT/dedup_full/pmc_$C" -o pmc --output-format csv \
    -- python3 bench.py --steps 2 --warmup 1 --no-cpu --components dedup --dedup-rows 100000000 \
    --dedup-full-rows 0 --no-explicit-rank --no-exchange-model > "$OUT/dedup_full_pmc_$C.log" 2>&1 || exit 1
done
python3 scripts/pmc_summary.py "$OUT/cas" "$OUT/pmc_cas.json" > "$OUT/pmc_cas.txt" || exit 1
python3 scripts/pmc_summary.py "$OUT/dedup" "$OUT/pmc_dedup.json" > "$OUT/pmc_dedup.txt" || exit 1
python3 scripts/pmc_summary.py "$OUT/dedup_full" "$OUT/pmc_dedup_full.json" > "$OUT/pmc_dedup_full.txt" || exit 1
python3 scripts/pmc_merge.py "$OUT" "$OUT/pmc_traffic.json" "$TAG" || exit 1
SD_BENCH_BACKEND=host timeout -k 10 600 python -u bench.py --gpus 2 --steps 3 --warmup 1 \
  --files 100000 --dedup-rows 2000000 --staged-files 50000 --staged-total-files 1000000 \
  --checksum-files 2 --checksum-bytes 268435456 --dir-files 1000 --no-cpu --verify \
  > "$OUT/rehearse2.json" 2> "$OUT/rehearse2.err" || exit 1
echo "exit 0"
