# Round 5 (historical: run on commit 1346212, where the LDS-staged group
# kernel k_bucket_group12_glds existed; it was removed after this A/B):
# correctness, then an interleaved A/B against SDGPU_GROUP_GLDS=0 at 100 M
# and 12.5 M rows (exp_seg_groups.py; the digest must match between legs).
#   TAG=r5n [TESTS=...] bash scripts/gpu_r5_glds.sh
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
  for g in 1 0 1 0; do
    SDGPU_GROUP_GLDS=$g timeout -k 10 120 python3 -u scripts/exp/exp_seg_groups.py $rows 20 \
      > gpurun_out/${TAG}_ab_tmp.json 2> gpurun_out/${TAG}_ab.err || { tail -5 gpurun_out/${TAG}_ab.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/${TAG}_ab_tmp.json')); d['GLDS']=$g; print(json.dumps(d))" \
      >> gpurun_out/${TAG}_ab.jsonl
    tail -1 gpurun_out/${TAG}_ab.jsonl | cut -c1-400
  done
done
