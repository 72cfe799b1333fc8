# A/B of config-1 staging on ONE box: slab = call / SDGPU_SLAB_DIV (6 or 10),
# tail taper SDGPU_SLAB_TAPER (0/1); three alternating rounds of the dir leg.
#   TAG=r4j bash scripts/gpu_r4_slab_ab.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for round in 1 2 3; do
  for cfg in "6 0" "6 1" "10 0" "10 1"; do
    set -- $cfg
    SDGPU_SLAB_DIV=$1 SDGPU_SLAB_TAPER=$2 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 \
      --no-cpu --components dir > gpurun_out/${TAG}_dir_d$1_t$2_$round.json 2> gpurun_out/${TAG}_dir_d$1_t$2_$round.err || exit 1
    python3 -c "
import json
d=json.loads(open('gpurun_out/${TAG}_dir_d$1_t$2_$round.json').read().strip().splitlines()[-1])['components']['dir']
p=d['phases_one_call']
print('round $round div $1 taper $2: %.0f files/s  fill %.2f ms  wait %.2f ms  slabs %d' % (d['value'], p['stage_fill']['ms'], p['stage_wait']['ms'], p['stage_fill']['n']))"
  done
done
