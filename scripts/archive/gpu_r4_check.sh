# Round-4 check: GPU tests (TESTS), then the driver's exact bench command.
#   TAG=r4a TESTS="tests/test_gpu_dedup.py ..." bash scripts/gpu_r4_check.sh
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
if [ -z "$NOBENCH" ]; then
  s=$(date +%s.%N)
  timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 ${BENCHARGS} \
    > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit 1
  e=$(date +%s.%N)
  python3 -c "print('bench wall s', $e - $s)"
  python3 scripts/bench_brief.py gpurun_out/${TAG}_bench.json
fi
