# A/B of the read-pool size on the config-1 directory leg (bench dir component).
# Usage: TAG=r3x bash scripts/gpu_r3_iothreads.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
cat /sys/fs/cgroup/cpu.max > gpurun_out/${TAG}_cpumax.txt 2>&1 || true
for T in 16 14 12 8 16; do
  SDGPU_IO_THREADS=$T timeout -k 10 200 python -u bench.py --components dir --steps 10 --warmup 1 --no-cpu \
    > gpurun_out/${TAG}_dir_t$T.json 2> gpurun_out/${TAG}_dir_t$T.err || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/${TAG}_dir_t$T.json'))['components']['dir']
print('threads $T', round(d['value']), 'files/s', round(d['ms_per_step'],2), 'ms/step, one call', round(d['phases_one_call']['call_ms'],2), 'ms, fill', round(d['phases_one_call']['stage_fill']['ms'],2))"
done
