# Round 5: SQ counters of the fused grouping's kernels at
# 100 M rows (two-level, k_bucket_group12_pk:ListOut) and 12.5 M rows, one
# rocprofv3 --pmc pass per counter set (no tracing in the same run).
#   TAG=r5m bash scripts/gpu_r5_pmc_group.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmcg_$TAG
mkdir -p "$OUT"
timeout -k 10 60 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || echo "counter list failed"
SETS=("SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
      "SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE GRBM_COUNT"
      "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_LDS_ATOMIC_RETURN SQ_INSTS_LDS_ATOMIC SQ_LDS_ADDR_CONFLICT SQ_INSTS_BRANCH")
for rows in 100000000 12500000; do
  i=0
  for C in "${SETS[@]}"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $C -d "$OUT/r${rows}_s$i" -o pmc --output-format csv \
      -- python3 scripts/exp/exp_seg_groups.py $rows 2 > "$OUT/r${rows}_s$i.log" 2>&1 \
      || { echo "set $i rows $rows failed"; tail -5 "$OUT/r${rows}_s$i.log"; }
  done
done
# the LDS-staged persistent variant (SDGPU_GROUP_GLDS=1, negative A/B; the
# knob existed until commit 1346212's kernel was removed), set 1
SDGPU_GROUP_GLDS=1 timeout -s KILL 120 rocprofv3 --pmc ${SETS[0]} -d "$OUT/glds_r12500000_s1" -o pmc \
  --output-format csv -- python3 scripts/exp/exp_seg_groups.py 12500000 2 > "$OUT/glds_s1.log" 2>&1 \
  || { echo "glds set failed"; tail -5 "$OUT/glds_s1.log"; }
python3 scripts/exp/pmc_kernels.py "$OUT" > "$OUT/summary.txt" || exit 1
cat "$OUT/summary.txt"
