set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rocm-smi --showproductname > gpurun_out/${TAG:-r1}_smi.txt 2>&1 || true
timeout -k 10 400 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG:-r1}_smoke.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG:-r1}_pytest.log 2>&1 && \
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 > gpurun_out/${TAG:-r1}_bench.json 2> gpurun_out/${TAG:-r1}_bench.err
echo "exit $?"
