# Latency-path check: the k_small parity tests plus the path drop-in tests,
# then the C-host single-file latency microbenchmark.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_latency.py tests/test_gpu_paths.py tests/test_gpu_checksum.py tests/test_gpu_cas.py \
  > gpurun_out/${TAG}_pytest.log 2>&1 || exit 1
timeout -k 10 120 ./build/exp_single_latency /tmp > gpurun_out/${TAG}_single.log 2>&1 || exit 1
echo "exit 0"
