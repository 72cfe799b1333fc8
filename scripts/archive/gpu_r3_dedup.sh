# Round-3 dedup change check: experiment binary (optional EXP), the grouping
# GPU tests, then the dedup component of the bench.  Usage:
#   TAG=r3x [EXP=exp_scatter_align] bash scripts/gpu_r3_dedup.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
if [ -n "$EXP" ]; then TAG=${TAG} EXP=$EXP bash scripts/gpu_r3_exp.sh 12500000 20 || exit 1; fi
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_dedup.py tests/test_gpu_fuzz.py tests/test_gpu_sharded.py tests/test_gpu_index.py \
  tests/test_gpu_job.py > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_pytest.log
[ $rc -eq 0 ] || { grep -n "FAILED\|Error" gpurun_out/${TAG}_pytest.log | head -20; exit $rc; }
timeout -k 10 300 python -u bench.py --components dedup --steps 10 --warmup 2 --no-cpu \
  > gpurun_out/${TAG}_dedup.json 2> gpurun_out/${TAG}_dedup.err || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/${TAG}_dedup.json'))['components']['dedup']
print('dedup 12.5M ms', d['ms_per_step'], {k: round(v['avg_ms'],4) for k,v in d['kernels'].items()})
f=d['config4_full_one_gpu']; print('100M ms', f['ms_per_step'], {k: round(v['avg_ms'],4) for k,v in f['kernels'].items()})"
