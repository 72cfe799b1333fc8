"""Experiment (not shipped): the config-1 identify call from Python under
different process settings (torch thread pool size, whether torch ran a CPU op
first), each in its own process, same files; prints median ms and the
library's stage_fill."""
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CHILD = r"""
import json, os, sys, time
import numpy as np
sys.path.insert(0, %r)
mode = sys.argv[1]
import torch
if mode == "threads1":
    torch.set_num_threads(1)
if mode in ("cpu_op", "threads1"):
    a = torch.randn(2000, 2000); (a @ a).sum().item()   # a parallel CPU op, as bench legs run
from spacedrive_amd import file_identifier as fi
from spacedrive_amd._native import default_context
d = json.load(open(%r))
paths, sizes = d["paths"], np.array(d["sizes"], np.uint64)
ctx = default_context(0)
fi.identify(paths, sizes=sizes, ctx=ctx)
ts = []
for _ in range(9):
    t0 = time.perf_counter(); fi.identify(paths, sizes=sizes, ctx=ctx); ts.append(time.perf_counter() - t0)
ctx.set_timing(True)
fi.identify(paths, sizes=sizes, ctx=ctx)
ph = {k: round(v[0], 2) for k, v in ctx.kernel_times().items() if k.startswith("stage")}
print(json.dumps({"mode": mode, "omp": os.environ.get("OMP_NUM_THREADS"), "median_ms": round(1e3 * sorted(ts)[4], 2), **ph}))
"""


def main():
    from spacedrive_amd import corpus
    root = tempfile.mkdtemp(prefix="direnv_")
    paths, sizes = corpus.write_config1_dir(root, 10000, seed=1)
    meta = os.path.join(root, "meta.json")
    json.dump({"paths": paths, "sizes": sizes.tolist()}, open(meta, "w"))
    for mode, omp in [("plain", None), ("cpu_op", None), ("threads1", None), ("cpu_op", "1"),
                      ("plain", None)]:
        env = dict(os.environ)
        if omp:
            env["OMP_NUM_THREADS"] = omp
        r = subprocess.run([sys.executable, "-c", CHILD % (ROOT, meta), mode], env=env,
                           capture_output=True, text=True, timeout=300)
        print(r.stdout.strip() or r.stderr[-1500:], flush=True)


if __name__ == "__main__":
    main()
