set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_paths.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_paths.log 2>&1 && \
timeout -k 10 300 python -u scripts/ab_k1.py 0,1 5 > gpurun_out/${TAG}_ab.log 2>&1 && \
timeout -k 10 700 python -u bench.py --steps ${STEPS:-5} --warmup 2 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
echo "exit $?"
