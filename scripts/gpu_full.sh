# Round checkpoint on one box: the whole GPU test suite,
# smoke, then the driver's exact bench command (wall-clocked).
#   TAG=r6x bash scripts/gpu_full.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests \
  > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_pytest.log
[ $rc -eq 0 ] || { grep -n "FAILED\|Error" gpurun_out/${TAG}_pytest.log | head -20; exit $rc; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -2 gpurun_out/${TAG}_smoke.log
s=$(date +%s.%N)
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 \
  > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit 1
e=$(date +%s.%N)
python3 -c "print('bench wall s', $e - $s)"
python3 scripts/bench_brief.py gpurun_out/${TAG}_bench.json
