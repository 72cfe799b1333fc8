# Bucket-partition block count A/B: dedup parity at two counts, then the dedup bench leg per count.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-pab}
for P in 256 100; do
  SDGPU_BUCKET_PART_BLOCKS=$P timeout -k 10 300 python -u -m pytest tests/test_gpu_dedup.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest_P$P.log 2>&1 || { echo "pytest P=$P failed"; exit 1; }
done
for P in ${PLIST:-256 128 512}; do
  SDGPU_BUCKET_PART_BLOCKS=$P timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --components dedup --no-cpu --files 100000 > gpurun_out/${T}_bench_P$P.json 2> gpurun_out/${T}_bench_P$P.err || { echo "bench P=$P failed"; exit 1; }
done
echo "exit 0"
