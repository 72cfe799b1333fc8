# A/B of the packed group kernel's L2 touch-ahead (SDGPU_GROUP_AHEAD=0 / 1):
# (Negative: the touch-ahead was removed after this A/B; logs in profiles/r4/ahead_ab/.)
# GPU tests of the grouping paths, then the dedup leg (12.5 M + 100 M rows,
# two-call and fused) with the touch off and on.
#   TAG=r4g bash scripts/gpu_r4_ahead.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_fused.py tests/test_gpu_dedup.py tests/test_gpu_sharded.py tests/test_gpu_index.py \
  > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?
tail -2 gpurun_out/${TAG}_pytest.log
[ $rc -eq 0 ] || { grep -n "FAILED\|Error" gpurun_out/${TAG}_pytest.log | head -20; exit $rc; }
for A in 0 1 0 1; do
  SDGPU_GROUP_AHEAD=$A timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu \
    --components dedup --no-exchange-model > gpurun_out/${TAG}_ahead$A.json 2> gpurun_out/${TAG}_ahead$A.err || exit 1
  echo "ahead=$A"; python3 scripts/bench_brief.py gpurun_out/${TAG}_ahead$A.json | grep -A4 "^dedup"
  cp gpurun_out/${TAG}_ahead$A.json gpurun_out/${TAG}_ahead${A}_$(date +%s).json
done
