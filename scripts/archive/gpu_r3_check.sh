# Round-3 check after a kernel change: the GPU tests of the touched kernels,
# then the bench components that time them.  Usage:
#   TAG=r3x TESTS="tests/test_gpu_dedup.py ..." COMPONENTS=dedup,consumers bash scripts/gpu_r3_check.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TESTS=${TESTS:-"tests/test_gpu_dedup.py tests/test_gpu_fuzz.py tests/test_gpu_stage_link.py tests/test_gpu_consumers.py tests/test_gpu_index.py tests/test_gpu_job.py"}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $TESTS \
  > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?
tail -2 gpurun_out/${TAG}_pytest.log
[ $rc -eq 0 ] || { grep -n "FAILED\|Error" gpurun_out/${TAG}_pytest.log | head -20; exit $rc; }
timeout -k 10 300 python -u bench.py --components ${COMPONENTS:-dedup,consumers} --steps 10 --warmup 2 --no-cpu \
  > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit 1
python3 - gpurun_out/${TAG}_bench.json <<'PY'
import json, sys
c = json.load(open(sys.argv[1]))["components"]
for name, v in c.items():
    if not isinstance(v, dict):
        continue
    ks = v.get("kernels") or {}
    print(name, v.get("ms_per_step"), {k: round(x["avg_ms"], 4) for k, x in ks.items()})
    for sub in ("config4_full_one_gpu", "link_batch", "orphan_remover", "thumbnail_shards"):
        s = v.get(sub)
        if isinstance(s, dict):
            print("  ", sub, s.get("ms_per_step"), {k: round(x["avg_ms"], 4) for k, x in (s.get("kernels") or {}).items()})
PY
