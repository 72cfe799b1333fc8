"""Diagnostic (round 6): the multi-process random call sequences of
tests/test_gpu_multiproc.py at W = 2 over many seeds, each rank's per-call
progress (SD_HOST_TRACE=1) written to gpurun_out/fuzz_desync/rank<r>.err, to
find a seed where the ranks' collective sequences part."""
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from oracle import oracle as O  # noqa: E402

world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
seeds = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else list(range(200, 285))
out_dir = os.path.join(ROOT, "gpurun_out", "fuzz_desync")
os.makedirs(out_dir, exist_ok=True)
work = tempfile.mkdtemp(prefix="sd_desync_")
CASES = ("uniform", "one_key_40k", "all_one_key")
TOTAL = 300_000
data = {}
for i, case in enumerate(CASES):
    rng = np.random.default_rng(300 + 7 * world + i)
    if case == "uniform":
        k, h, _ = O.synth_dedup_rows(300 + 7 * world + i, TOTAL, int(TOTAL * 0.8), 0, TOTAL)
    else:
        pool = rng.integers(0, 2**64 - 1, TOTAL, dtype=np.uint64, endpoint=True)
        k = pool[rng.integers(0, pool.size // 2, TOTAL)]
        if case == "one_key_40k":
            k[rng.choice(TOTAL, 40_000, replace=False)] = pool[7]
        else:
            k[:] = pool[7]
        h = (rng.random(TOTAL) > 0.01).astype(np.uint8)
    sp = np.array([(TOTAL * r * (r + 1) // (world * (world + 1)),
                    TOTAL * (r + 1) * (r + 2) // (world * (world + 1))) for r in range(world)], np.int64)
    data[f"k_{case}"], data[f"h_{case}"], data[f"span_{case}"] = k, h, sp
    data[f"B_{case}"] = np.int64((sp[:, 1] - sp[:, 0]).max())
data["cases"] = np.array(CASES)
data["fuzz_ops"] = np.int64(20)
data["msg_bytes"] = np.int64(16 * world * (TOTAL + 4096))
np.savez(os.path.join(work, "data.npz"), **data)
env = dict(os.environ, SD_HOST_TIMEOUT_MS="20000", SD_HOST_TRACE="1")
reps = int(os.environ.get("SD_DESYNC_REPS", "1"))
for rep in range(reps):  # until the first failure
    wdir = tempfile.mkdtemp(prefix="sd_desync_run_")
    os.symlink(os.path.join(work, "data.npz"), os.path.join(wdir, "data.npz"))
    procs = []
    for r in range(world):
        err = open(os.path.join(out_dir, f"rank{r}.err"), "w")
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.join(ROOT, "tests", "_host_rank.py"),
                                       ROOT, str(world), str(r), wdir,
                                       ",".join(f"fuzz_{s}" for s in seeds)],
                                      stdout=subprocess.DEVNULL, stderr=err, env=env))
    rcs = [p.wait(timeout=900) for p in procs]
    print("rep", rep, "rank exit codes", rcs, flush=True)
    if any(rcs):
        break
