# Round-3 checkpoint on one GPU box: the whole -m gpu suite, smoke(), then the
# driver's exact bench command with its wall clock.  Usage:
#   TAG=r3x bash scripts/gpu_r3_full.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -x build/exp_uring ] && [ -z "$NO_URING_AB" ]; then TAG=${TAG} bash scripts/gpu_r3_uring_ab.sh || true; fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit 1
TAG=${TAG} bash scripts/gpu_r3_rehearse.sh
