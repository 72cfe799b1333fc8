# Round-3 quick check: the GPU tests of the files changed this round, then the
# experiment binaries with their profiles.  Usage: TAG=r3x bash scripts/gpu_r3_quick.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG} EXP=exp_xcd_scatter bash scripts/gpu_r3_exp.sh 12500000 20 || exit 1
TAG=${TAG} EXP=exp_group_packed bash scripts/gpu_r3_exp.sh 12500000 20 || exit 1
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_latency.py tests/test_gpu_sharded.py tests/test_gpu_index.py \
  tests/test_gpu_stage_link.py > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?
tail -5 gpurun_out/${TAG}_pytest.log
[ $rc -eq 0 ] || { grep -n "FAILED\|Error\|error" gpurun_out/${TAG}_pytest.log | head -20; exit $rc; }
