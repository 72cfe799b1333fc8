# The N > 1 identifier step rehearsed on one GPU: the job's grouping through a
# one-rank RCCL communicator (sharded path + link batch) vs the N = 1 fused
# call, same box, alternating.
#   TAG=r4n bash scripts/gpu_r4_forcecomm.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for round in 1 2; do
  for F in 0 1; do
    SD_BENCH_FORCE_COMM=$F timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu \
      --components cas > gpurun_out/${TAG}_fc${F}_$round.json 2> gpurun_out/${TAG}_fc${F}_$round.err || exit 1
    python3 -c "
import json
d=json.loads(open('gpurun_out/${TAG}_fc${F}_$round.json').read().strip().splitlines()[-1])
c=d['components']
print('round $round force_comm $F: job %.3f ms  cas %.3f ms  grouping %s  world %s' % (c['identifier_job']['ms_per_step'], c['cas']['ms_per_step'], c['identifier_job'].get('grouping'), d['world'].get('rccl', {}).get('stats_rank')))"
  done
done
