# Round 5: the grouping A/B used for every group-kernel and partition change
# of the round (first written for the leaner packed group kernel).  Optional
# GPU tests, then an A/B against a build of the previous tree
# (build/ab/libsdgpu_prev.so, AB_LIB) at 100 M and 12.5 M rows, alternating
# processes, then SQ counters of the group kernel.
#   TAG=r5q [TESTS=...] bash scripts/gpu_r5_pk.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $TESTS \
    > gpurun_out/${TAG}_pytest.log 2>&1
  rc=$?
  tail -2 gpurun_out/${TAG}_pytest.log
  [ $rc -eq 0 ] || { grep -n "FAILED\|Error" gpurun_out/${TAG}_pytest.log | head -20; exit $rc; }
fi
for rows in 100000000 12500000; do
  for lib in build/ab/libsdgpu_prev.so "" build/ab/libsdgpu_prev.so ""; do
    AB_LIB=$lib timeout -k 10 120 python3 -u scripts/exp/exp_seg_groups.py $rows 20 \
      > gpurun_out/${TAG}_ab_tmp.json 2> gpurun_out/${TAG}_ab.err || { tail -5 gpurun_out/${TAG}_ab.err; exit 1; }
    cat gpurun_out/${TAG}_ab_tmp.json >> gpurun_out/${TAG}_ab.jsonl
    tail -1 gpurun_out/${TAG}_ab.jsonl | cut -c1-420
  done
done
OUT=gpurun_out/pmcg_$TAG
mkdir -p "$OUT"
S1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
S2="SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE GRBM_COUNT"
for rows in 100000000 12500000; do
  i=0
  for C in "$S1" "$S2"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $C -d "$OUT/r${rows}_s$i" -o pmc --output-format csv \
      -- python3 scripts/exp/exp_seg_groups.py $rows 2 > "$OUT/r${rows}_s$i.log" 2>&1 \
      || { echo "set $i rows $rows failed"; tail -5 "$OUT/r${rows}_s$i.log"; }
  done
done
python3 scripts/exp/pmc_kernels.py "$OUT" > "$OUT/summary.txt" || exit 1
grep -A1 "==\|group12" "$OUT/summary.txt" | cut -c1-400
