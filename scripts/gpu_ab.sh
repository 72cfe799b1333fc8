set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/ab_k1.py ${AB:-0,2} 5 > gpurun_out/${TAG}_ab.log 2>&1
echo "exit $?"
