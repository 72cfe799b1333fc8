# Multi-rank rehearsal of bench.py on ONE GPU (run via gpurun): N processes share
# the card, the grouping exchange goes over gloo (host) instead of RCCL, and
# --verify checks the sharded grouping against the one-GPU grouping.  Exercises
# every rank-dependent branch of bench.py (seeds, global ranks, rank-0-only CPU
# baseline, barriers, max-over-ranks) without an 8-GPU node.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${TAG:-reh}
export SD_BENCH_BACKEND=gloo
run() {  # run <nproc> <port> <bench args...>
  local n=$1 port=$2; shift 2
  timeout -k 10 420 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" \
    --master-addr 127.0.0.1 --master-port "$port" bench.py --gpus "$n" "$@" \
    > "gpurun_out/${T}_w${n}.json" 2> "gpurun_out/${T}_w${n}.err"
}
run 2 29511 --steps 3 --warmup 1 --verify --files 500000 --checksum-files 8 --cpu-seconds 3 \
  || { echo "world 2 failed: $?"; exit 1; }
run 4 29512 --steps 2 --warmup 1 --verify --files 200000 --dedup-rows 4000000 \
  --checksum-files 2 --staged-files 50000 --dir-files 2000 --no-cpu \
  || { echo "world 4 failed: $?"; exit 1; }
echo "exit 0"
