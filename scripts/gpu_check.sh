# GPU check: the GPU tests named in TESTS (default: all), then optionally a
# short bench (BENCH=1, BENCHARGS) -- each step under its own time limit,
# chained so that a failure ends the call.
#   TAG=r6a TESTS="tests/test_gpu_multiproc.py" [BENCH=1 BENCHARGS="--components dedup"] \
#     bash scripts/gpu_check.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 ${TEST_LIMIT:-900} python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  -m gpu ${TESTS:-tests} > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_pytest.log
[ $rc -eq 0 ] || { grep -n "FAILED\|Error" gpurun_out/${TAG}_pytest.log | head -20; exit $rc; }
if [ -n "$BENCH" ]; then
  timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 ${BENCHARGS} \
    > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit 1
  python3 scripts/bench_brief.py gpurun_out/${TAG}_bench.json
fi
