# Parity suite + the cheap bench legs (cas, single-file latency, config-1 dir).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-q}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { echo "pytest failed"; exit 1; }
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --components ${COMPS:-cas,single,dir} --no-cpu > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo "bench failed"; exit 1; }
echo "exit 0"
