# Round-2 GPU bench: default N=1 bench, then a 2-rank gloo rehearsal through
# bench.py's own --gpus self-launch (one GPU box).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit 1
SD_BENCH_BACKEND=gloo timeout -k 10 600 python -u bench.py --gpus 2 --steps 3 --warmup 1 \
  --files 100000 --dedup-rows 2000000 --staged-files 50000 --staged-total-files 1000000 \
  --checksum-files 2 --checksum-bytes 268435456 --dir-files 1000 --no-cpu --verify \
  > gpurun_out/${TAG}_rehearse2.json 2> gpurun_out/${TAG}_rehearse2.err || exit 1
echo "exit 0"
