# A/B: the orphan remover's mark ranges (SDGPU_MARK_RANGES 8/4/2/1: fewer
# (Done: 8 ranges kept, the knob removed; logs in profiles/r4/consumers_ab/.)
# re-reads of the file_path ids vs L2-local marking), with the consumer tests
# under each; then the config-1 directory leg (staging slabs of a tenth).
#   TAG=r4i bash scripts/gpu_r4_consumers_ab.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for R in 8 4 2 1; do
  SDGPU_MARK_RANGES=$R timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    -m gpu tests/test_gpu_consumers.py > gpurun_out/${TAG}_pytest_r$R.log 2>&1 || { tail -5 gpurun_out/${TAG}_pytest_r$R.log; exit 1; }
  tail -1 gpurun_out/${TAG}_pytest_r$R.log
  SDGPU_MARK_RANGES=$R timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu \
    --components consumers > gpurun_out/${TAG}_cons_r$R.json 2> gpurun_out/${TAG}_cons_r$R.err || exit 1
  python3 -c "
import json
d=json.loads(open('gpurun_out/${TAG}_cons_r$R.json').read().strip().splitlines()[-1])['components']['consumers']
print('ranges $R orphan_remover ms', round(d['orphan_remover']['ms_per_step'],4), 'thumbnail ms', round(d['thumbnail_shards']['ms_per_step'],4))"
done
for k in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --components cas,dir \
    > gpurun_out/${TAG}_dir$k.json 2> gpurun_out/${TAG}_dir$k.err || exit 1
  python3 -c "
import json
d=json.loads(open('gpurun_out/${TAG}_dir$k.json').read().strip().splitlines()[-1])
print('dir', round(d['components']['dir']['value']), 'cpu', round(d['cpu_baseline']['config1_dir']['value']), json.dumps(d['components']['dir']['phases_one_call']))"
done
