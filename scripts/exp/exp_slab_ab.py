"""Experiment (round 6): config-1 staging-slab sizing A/B
on ONE box, variants alternating process by process so box-to-box noise (the
fill swings 10.5-14.8 ms across boxes) cancels.  Each child: one warm call,
then 40 timed sdgpu_identify_files calls over the same 10 k-file directory,
median and the library's stage phases of one more call.
Variants: SDGPU_SLAB_DIV (slab = call bytes / div, default 6),
SDGPU_SLAB_TAPER (last slabs shrink geometrically), and the process pinned to
one NUMA node's CPUs (node0 / node1), and the read-pool size (io15 / io14 /
io12: SDGPU_IO_THREADS; default min(16, cgroup CPU quota)).
Usage: python scripts/exp/exp_slab_ab.py [rounds] [variant,variant,...]"""
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

CHILD = r"""
import json, os, sys, time
import numpy as np
node = os.environ.get("SD_AB_NODE")
if node is not None:  # pin this process (the read pool inherits it) to one NUMA node's CPUs
    cpus = set()
    for part in open(f"/sys/devices/system/node/node{node}/cpulist").read().strip().split(","):
        lo, _, hi = part.partition("-")
        cpus.update(range(int(lo), int(hi or lo) + 1))
    os.sched_setaffinity(0, cpus & os.sched_getaffinity(0))
sys.path.insert(0, %r)
from spacedrive_amd import file_identifier as fi
from spacedrive_amd._native import default_context
d = json.load(open(%r))
paths, sizes = fi.PathList(d["paths"]), np.array(d["sizes"], np.uint64)
ctx = default_context(0)
fi.identify(paths, sizes=sizes, ctx=ctx)
ts = []
for _ in range(40):
    t0 = time.perf_counter(); r = fi.identify(paths, sizes=sizes, ctx=ctx); ts.append(time.perf_counter() - t0)
assert (r.status == 0).all()
ctx.set_timing(True)
fi.identify(paths, sizes=sizes, ctx=ctx)
ph = {k: round(v[0], 3) for k, v in ctx.kernel_times().items()}
ts.sort()
print(json.dumps({"median_ms": round(1e3 * ts[20], 3), "p25_ms": round(1e3 * ts[10], 3),
                  "digest": int(np.bitwise_xor.reduce(r.cas8.view(np.uint64).ravel())), **ph}))
"""

ALL = {"div6": {}, "div12": {"SDGPU_SLAB_DIV": "12"}, "div16": {"SDGPU_SLAB_DIV": "16"},
       "div24": {"SDGPU_SLAB_DIV": "24"},
       "div6_taper": {"SDGPU_SLAB_TAPER": "1"},
       "div12_taper": {"SDGPU_SLAB_DIV": "12", "SDGPU_SLAB_TAPER": "1"},
       "node0": {"SD_AB_NODE": "0"}, "node1": {"SD_AB_NODE": "1"},
       "io15": {"SDGPU_IO_THREADS": "15"}, "io14": {"SDGPU_IO_THREADS": "14"},
       "io12": {"SDGPU_IO_THREADS": "12"}}


def topology():
    """CPUs this process may use, NUMA nodes, and the GPU's node."""
    out = {"affinity": len(os.sched_getaffinity(0))}
    base = "/sys/devices/system/node"
    for d in sorted(os.listdir(base)) if os.path.isdir(base) else []:
        if d.startswith("node") and d[4:].isdigit():
            out[d] = open(f"{base}/{d}/cpulist").read().strip()
    try:
        for dev in sorted(os.listdir("/sys/class/drm")):
            p = f"/sys/class/drm/{dev}/device/numa_node"
            if dev.startswith("card") and "-" not in dev and os.path.exists(p):
                out[f"{dev}_numa"] = open(p).read().strip()
    except OSError:
        pass
    try:
        out["cpu.max"] = open("/sys/fs/cgroup/cpu.max").read().strip()
    except OSError:
        pass
    return out


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    names = sys.argv[2].split(",") if len(sys.argv) > 2 else ["div6", "div12", "div6_taper",
                                                              "div12_taper"]
    VARIANTS = [(n, ALL[n]) for n in names]
    print(json.dumps(topology()), flush=True)
    from spacedrive_amd import corpus
    root = tempfile.mkdtemp(prefix="slab_ab_")
    paths, sizes = corpus.write_config1_dir(root, 10000, seed=1)
    os.sync()
    meta = os.path.join(root, "meta.json")
    json.dump({"paths": paths, "sizes": sizes.tolist()}, open(meta, "w"))
    res = {name: [] for name, _ in VARIANTS}
    for rd in range(rounds):
        order = VARIANTS if rd % 2 == 0 else VARIANTS[::-1]
        for name, env_add in order:
            env = dict(os.environ, **env_add)
            r = subprocess.run([sys.executable, "-c", CHILD % (ROOT, meta)], env=env,
                               capture_output=True, text=True, timeout=120)
            if r.returncode != 0:
                print(name, "failed:", r.stderr[-1500:], flush=True)
                sys.exit(1)
            out = json.loads(r.stdout.strip().splitlines()[-1])
            out["variant"], out["round"] = name, rd
            res[name].append(out)
            print(json.dumps(out), flush=True)
    digests = {o["digest"] for v in res.values() for o in v}
    for name, v in res.items():
        med = sorted(o["median_ms"] for o in v)
        print(f"{name:12s} median-of-medians {med[len(med) // 2]:.3f} ms  all {med}", flush=True)
    print("digests equal:", len(digests) == 1, flush=True)


if __name__ == "__main__":
    main()
