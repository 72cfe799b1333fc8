# dedup check then the full checkpoint (one box).  Usage: TAG=r3x bash scripts/gpu_r3_all.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${TAG}_d bash scripts/gpu_r3_dedup.sh || exit 1
TAG=${TAG} bash scripts/gpu_r3_full.sh
