# A/B: the list-writing group kernel's in-bucket ranks -- workgroup ranks
# (Done: atomic ranks adopted as the only ListOut, the knob removed; profiles/r4/listranks_ab/.)
# (ListOut, two barriers + a one-wave scan) vs one LDS atomic per wave
# (ListOutA, SDGPU_LIST_RANKS=atomic); the fused-path tests under the atomic
# variant, then the dedup leg alternating.
#   TAG=r4k bash scripts/gpu_r4_listranks_ab.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
SDGPU_LIST_RANKS=atomic timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  -m gpu tests/test_gpu_fused.py > gpurun_out/${TAG}_pytest_atomic.log 2>&1 || { tail -5 gpurun_out/${TAG}_pytest_atomic.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest_atomic.log
for round in 1 2; do
  for V in wg atomic; do
    SDGPU_LIST_RANKS=$V timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu \
      --components dedup --no-exchange-model > gpurun_out/${TAG}_lr_${V}_$round.json 2> gpurun_out/${TAG}_lr_${V}_$round.err || exit 1
    python3 -c "
import json
c=json.loads(open('gpurun_out/${TAG}_lr_${V}_$round.json').read().strip().splitlines()[-1])['components']['dedup']
f=c['fused_job']; g=c['config4_full_one_gpu']['fused_job']
print('round $round ranks $V: 12.5M fused %.4f ms (group %.4f)  100M fused %.4f ms (group %.4f)' % (f['ms_per_step'], f['kernels']['bucket_group']['avg_ms'], g['ms_per_step'], g['kernels']['bucket_group']['avg_ms']))"
  done
done
