# Rehearses the driver's round-end bench command on the current tree and
# records its wall clock.  Usage (on the GPU box):
#   TAG=r3a bash scripts/gpu_r3_rehearse.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${TAG:-r3}
t0=$(date +%s.%N)
timeout -k 10 560 python3 bench.py --gpus 1 --steps 20 --warmup 5 \
  > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
rc=$?
t1=$(date +%s.%N)
python3 - "$t0" "$t1" "$rc" > gpurun_out/${T}_bench_wall.json <<'EOF'
import json, sys
t0, t1, rc = float(sys.argv[1]), float(sys.argv[2]), int(sys.argv[3])
print(json.dumps({"cmd": "python3 bench.py --gpus 1 --steps 20 --warmup 5",
                  "wall_s": round(t1 - t0, 1), "rc": rc}))
EOF
cat gpurun_out/${T}_bench_wall.json
exit $rc
