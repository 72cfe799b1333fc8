# Full GPU cycle: parity suite -> K1 A/B -> bench -> rocprofv3 kernel trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-rx}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { echo "pytest failed"; exit 1; }
if [ -n "$AB" ]; then timeout -k 10 300 python -u scripts/ab_k1.py $AB 5 > gpurun_out/${T}_ab.log 2>&1 || exit 1; fi
timeout -k 10 700 python -u bench.py --steps ${STEPS:-5} --warmup 2 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo "bench failed"; exit 1; }
if [ -n "$PROF" ]; then TAG=$T bash scripts/profile.sh > gpurun_out/${T}_prof.log 2>&1 || { echo "profile failed"; exit 1; }; fi
echo "exit 0"
