# io_uring vs pread A/B for the config-1 staging reads, on
# the GPU box's host (CPU only; the box's kernel, filesystem and CPU share are
# what the dir leg runs on).  build/exp_uring is built from scripts/exp/exp_uring.cpp.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${TAG:-r3}
D=$(mktemp -d /tmp/sd_cfg1_ab_XXXX)
python3 - "$D" > "$D.lst" <<'PY'
import sys
sys.path.insert(0, ".")
from spacedrive_amd import corpus
paths, sizes = corpus.write_config1_dir(sys.argv[1], 10000, seed=1)
for p, s in zip(paths, sizes):
    print(int(s), p)
PY
{ nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; uname -r; df -T /tmp | tail -1; } > gpurun_out/${T}_uring_env.txt
timeout -k 10 120 build/exp_uring "$D.lst" 16 3 > gpurun_out/${T}_uring_ab.log 2>&1
rc=$?
timeout -k 10 120 build/exp_uring "$D.lst" 1 2 >> gpurun_out/${T}_uring_ab.log 2>&1
rm -rf "$D" "$D.lst"
cat gpurun_out/${T}_uring_ab.log
exit $rc
