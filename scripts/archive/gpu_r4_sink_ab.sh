# A/B: keyless rows of the fused grouping collected by the first partition
# pass (default) vs the separate extra-entry pass (SDGPU_KEYLESS_PASS=1), the
# fused tests under both, then the dedup leg alternating (one box).
#   TAG=r4x bash scripts/gpu_r4_sink_ab.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_fused.py > gpurun_out/${TAG}_pytest_sink.log 2>&1 \
  || { tail -30 gpurun_out/${TAG}_pytest_sink.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest_sink.log
SDGPU_KEYLESS_PASS=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_fused.py > gpurun_out/${TAG}_pytest_pass.log 2>&1 \
  || { tail -30 gpurun_out/${TAG}_pytest_pass.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest_pass.log
for round in 1 2 3; do
  for V in 0 1; do
    SDGPU_KEYLESS_PASS=$V timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu \
      --no-exchange-model --no-explicit-rank --components dedup \
      > gpurun_out/${TAG}_dedup_${V}_$round.json 2> gpurun_out/${TAG}_dedup_${V}_$round.err || exit 1
    python3 -c "
import json
d=json.loads(open('gpurun_out/${TAG}_dedup_${V}_$round.json').read().strip().splitlines()[-1])['components']['dedup']
f=d['fused_job']; g=d['config4_full_one_gpu']['fused_job']
k=lambda x: ' '.join('%s %.4f' % (a, b['avg_ms']) for a, b in x['kernels'].items())
print('round $round pass=$V: 12.5M %.4f ms [%s] | 100M %.4f ms mism %s [%s]' % (f['ms_per_step'], k(f), g['ms_per_step'], g.get('list_mismatches_vs_oracle'), k(g)))"
  done
done
