# Round 5: A/B of libsdgpu builds (AB_LIB; "tree" = the tree's own) on the fused
# grouping (scripts/exp/exp_seg_groups.py), alternating processes.
#   TAG=r5v ROWS="100000000" LIBS="build/ab/libsdgpu_prev.so tree" bash scripts/gpu_r5_ab.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for rows in ${ROWS:-100000000}; do
  for rep in 1 2; do
    for lib in $LIBS; do
      [ "$lib" = tree ] && lib=""
      AB_LIB=$lib timeout -k 10 120 python3 -u scripts/exp/exp_seg_groups.py $rows 20 \
        > gpurun_out/${TAG}_ab_tmp.json 2> gpurun_out/${TAG}_ab.err || { tail -5 gpurun_out/${TAG}_ab.err; exit 1; }
      cat gpurun_out/${TAG}_ab_tmp.json >> gpurun_out/${TAG}_ab.jsonl
      python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_ab_tmp.json')); print(d['lib'], d['rows'], round(d['ms_per_call'],4), {k: round(v,4) for k, v in d['kernels'].items()}, d['digest'][:10])"
    done
  done
done
