# A/B: ring staging of sdgpu_identify_files (SDGPU_STAGE=ring: small hot
# (Negative: ring staging removed after this A/B; logs in profiles/r4/ring_ab/.)
# pinned buffers copied H2D into a device arena, K1 per segment) against the
# slab pipeline; the path tests under ring staging first, then the config-1
# directory leg alternating (one box), then the small-copy H2D experiment.
#   TAG=r4v bash scripts/gpu_r4_ring_ab.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
SDGPU_STAGE=ring timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_job.py tests/test_gpu_paths.py tests/test_gpu_burst.py > gpurun_out/${TAG}_pytest_ring.log 2>&1 \
  || { tail -30 gpurun_out/${TAG}_pytest_ring.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest_ring.log
for round in 1 2 3; do
  for S in slab ring; do
    SDGPU_STAGE=$S timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu --components dir \
      > gpurun_out/${TAG}_dir_${S}_$round.json 2> gpurun_out/${TAG}_dir_${S}_$round.err || exit 1
    python3 -c "
import json
d=json.loads(open('gpurun_out/${TAG}_dir_${S}_$round.json').read().strip().splitlines()[-1])['components']['dir']
p=d['phases_one_call']
print('round $round $S: %.0f files/s  fill %.2f ms  wait %.2f ms  call %.2f ms' % (d['value'], p['stage_fill']['ms'], p['stage_wait']['ms'], p['call_ms']))"
  done
done
timeout -k 10 180 build/exp_h2d_small > gpurun_out/${TAG}_h2d.log 2>&1 && cat gpurun_out/${TAG}_h2d.log
