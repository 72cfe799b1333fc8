# Latency service check: its GPU tests, then the bench's single-file leg alone.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG} EXP=exp_scatter_align bash scripts/gpu_r3_exp.sh 12500000 20 || exit 1
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_latency.py tests/test_gpu_paths.py > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
timeout -k 10 300 python -u bench.py --components single --steps 3 --warmup 1 --no-cpu \
  > gpurun_out/${TAG}_single.json 2> gpurun_out/${TAG}_single.err || exit 1
python3 -c "import json; print(json.dumps(json.load(open('gpurun_out/${TAG}_single.json'))['components']['single_file_latency'], indent=1))"
# config 5 on disk (200 k sparse config-2 files), pread and io_uring staging
df -h /tmp | tail -1
timeout -k 10 400 python -u scripts/disk_identify.py --files 200000 > gpurun_out/${TAG}_disk_pread.json 2> gpurun_out/${TAG}_disk_pread.err || exit 1
cat gpurun_out/${TAG}_disk_pread.json
SDGPU_IO=uring timeout -k 10 400 python -u scripts/disk_identify.py --files 200000 > gpurun_out/${TAG}_disk_uring.json 2> gpurun_out/${TAG}_disk_uring.err || exit 1
cat gpurun_out/${TAG}_disk_uring.json
