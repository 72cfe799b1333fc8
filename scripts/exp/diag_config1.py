"""Config-1 diagnostic: where the pinned-slab fill of sdgpu_identify_files
spends its time on a given box.  Prints the process's CPU set and NUMA nodes,
then per call: the wall time and the library's phase timers (fill = the pool's
preads into the pinned slabs).  SDGPU_IO_THREADS is read once per process, so
each thread count runs as its own process (scripts/exp/diag_config1.sh).
  python3 scripts/exp/diag_config1.py <dir> [calls]
"""
import glob
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from spacedrive_amd import corpus, file_identifier as fi  # noqa: E402
from spacedrive_amd._native import default_context  # noqa: E402


def nodes_of(cpus):
    out = {}
    for d in sorted(glob.glob("/sys/devices/system/node/node[0-9]*")):
        lst = open(os.path.join(d, "cpulist")).read().strip()
        s = set()
        for part in lst.split(","):
            if "-" in part:
                a, b = part.split("-")
                s.update(range(int(a), int(b) + 1))
            elif part:
                s.add(int(part))
        k = len(s & cpus)
        if k:
            out[os.path.basename(d)] = k
    return out


def main():
    root = sys.argv[1]
    calls = int(sys.argv[2]) if len(sys.argv) > 2 else 9
    os.makedirs(root, exist_ok=True)
    marker = os.path.join(root, ".done")
    if not os.path.exists(marker):
        paths, sizes = corpus.write_config1_dir(root, 10_000, seed=1)
        os.sync()
        json.dump({"paths": paths, "sizes": [int(x) for x in sizes]}, open(marker, "w"))
    m = json.load(open(marker))
    paths, sizes = fi.PathList(m["paths"]), np.array(m["sizes"], np.uint64)
    ctx = default_context()
    cpus = os.sched_getaffinity(0)
    info = {"io": os.environ.get("SDGPU_IO", "pread"), "io_threads_env": os.environ.get("SDGPU_IO_THREADS"), "cpus": len(cpus),
            "nodes": nodes_of(cpus), "bytes": None}
    fi.identify(paths, sizes=sizes, ctx=ctx)  # warm
    ts, fills = [], []
    for _ in range(calls):
        ctx.set_timing(True)
        t = time.perf_counter()
        fi.identify(paths, sizes=sizes, ctx=ctx)
        ts.append(1e3 * (time.perf_counter() - t))
        ph = ctx.kernel_times()
        ctx.set_timing(False)
        fills.append(ph.get("stage_fill", (0, 0))[0])
    info.update({"call_ms": [round(x, 2) for x in ts], "fill_ms": [round(x, 2) for x in fills],
                 "median_call_ms": float(np.median(ts)), "median_fill_ms": float(np.median(fills))})
    print(json.dumps(info))


if __name__ == "__main__":
    main()
