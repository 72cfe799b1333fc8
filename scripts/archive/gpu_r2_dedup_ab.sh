# Dedup change check: grouping/index/job GPU tests, then the dedup component
# of the bench (12.5 M rows + 100 M rows on one GPU).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_dedup.py tests/test_gpu_sharded.py tests/test_gpu_index.py tests/test_gpu_job.py \
  > gpurun_out/${TAG}_pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --components dedup --steps 10 --warmup 2 --no-cpu \
  > gpurun_out/${TAG}_dedup.json 2> gpurun_out/${TAG}_dedup.err || exit 1
echo "exit 0"
