set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_job.py tests/test_gpu_paths.py > gpurun_out/r5io_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r5io_pytest.log; [ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/diag_config1.jsonl
bash scripts/exp/diag_config1.sh
