# Exchange path check: sharded/dedup GPU tests, then a one-rank bench through
# libsdgpu's RCCL communicator (stdout must hold exactly one JSON line).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_sharded.py tests/test_gpu_dedup.py > gpurun_out/${TAG}_pytest.log 2>&1 || exit 1
SD_BENCH_FORCE_COMM=1 timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 --no-cpu \
  --staged-total-files 5000000 > gpurun_out/${TAG}_comm.json 2> gpurun_out/${TAG}_comm.err || exit 1
echo "exit 0"
