# Config-1 fill diagnostic on one box: the same 10 k-file directory read by
# the pread pool, the bounce-buffer reader (SDGPU_IO=bounce) and io_uring at
# 16 / 8 pool threads (one process each), plus the CPU set and NUMA nodes.
# Output: gpurun_out/diag_config1.jsonl
#   bash scripts/exp/diag_config1.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
D=$(mktemp -d /tmp/sd_diag_XXXX)
for cfg in "16 pread" "16 bounce" "16 uring" "16 pread" "16 bounce" "8 bounce"; do set -- $cfg; t=$1; io=$2
  SDGPU_IO=$io SDGPU_IO_THREADS=$t timeout -k 10 120 python3 -u scripts/exp/diag_config1.py "$D" 9 \
    >> gpurun_out/diag_config1.jsonl 2> gpurun_out/diag_config1.err || { tail -5 gpurun_out/diag_config1.err; exit 1; }
  tail -1 gpurun_out/diag_config1.jsonl
done
rm -rf "$D"
