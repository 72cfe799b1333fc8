# Round 5: GPU tests (TESTS) then the exchange timelines (gpu_r5_xtrace.sh).
#   TAG=r5e TESTS="..." bash scripts/gpu_r5_combo.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $TESTS \
    > gpurun_out/${TAG}_pytest.log 2>&1
  rc=$?
  tail -2 gpurun_out/${TAG}_pytest.log
  [ $rc -eq 0 ] || { grep -n "FAILED\|Error" gpurun_out/${TAG}_pytest.log | head -20; exit $rc; }
fi
bash scripts/gpu_r5_xtrace.sh
