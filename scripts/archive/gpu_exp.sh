set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for x in ${EXPS:-exp_sdwa}; do timeout -k 10 120 ./build/$x > gpurun_out/${TAG}_$x.log 2>&1 || exit 1; done
echo "exit 0"
