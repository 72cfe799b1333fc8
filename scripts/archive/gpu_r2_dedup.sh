export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_index.py tests/test_gpu_sharded.py tests/test_gpu_dedup.py -x -v --timeout 400 --timeout-method thread > gpurun_out/r2_dedup.log 2>&1 && \
timeout -k 10 300 python -u bench.py --components dedup --steps 10 --warmup 3 --no-cpu --files 200000 > gpurun_out/r2_bench_dedup.json 2> gpurun_out/r2_bench_dedup.err
