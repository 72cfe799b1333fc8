# Round 5: A/B of SDGPU_SEG_GROUPS (two-level second pass + group kernel per
# group of coarse segments) on the fused 100 M-row call, then the counter list.
#   TAG=r5j bash scripts/gpu_r5_seggroups.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/seg_$TAG
mkdir -p "$OUT"
for G in ${GS:-1 2 4 8 16 1}; do
  SDGPU_SEG_GROUPS=$G timeout -k 10 200 python3 scripts/exp/exp_seg_groups.py 100000000 20 \
    >> "$OUT/ab.jsonl" 2>> "$OUT/ab.err" || exit 1
  tail -1 "$OUT/ab.jsonl" | cut -c1-400
done
timeout -k 10 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
