# Dedup kernels: parity of the grouping / link tests, then the cas + dedup bench legs.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-dd}
timeout -k 10 300 python -u -m pytest tests/test_gpu_dedup.py tests/test_gpu_stage_link.py tests/test_gpu_paths.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { echo "pytest failed"; exit 1; }
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --components cas,dedup --no-cpu > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo "bench failed"; exit 1; }
echo "exit 0"
