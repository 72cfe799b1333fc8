"""Runs tests/_host_rank.py scenarios at a given world size on the data the
multi-process test uses (diagnostics; prints every rank's JSON lines).

    python scripts/exp/exp_multiproc_probe.py <world> <scenario,...>
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import json
    import tempfile
    import numpy as np
    import test_gpu_multiproc as T
    from oracle import oracle as O
    world, scenarios = int(sys.argv[1]), sys.argv[2].split(",")
    work = tempfile.mkdtemp(prefix=f"sd_probe{world}_")
    data = {}
    for i, case in enumerate(T.CASES):
        k, h = T._rows(case, T.TOTAL, 90 + 7 * world + i)
        sp = T._spans(T.TOTAL, world)
        data[f"k_{case}"], data[f"h_{case}"], data[f"span_{case}"] = k, h, sp
        data[f"B_{case}"] = np.int64((sp[:, 1] - sp[:, 0]).max())
        ref = O.group_reps(k, h, 100)
        c, lr, lo = O.link_batch(ref, None, np.ones(T.TOTAL, np.uint8), 0)
        print(json.dumps({"case": case, "spans": sp.tolist(), "creators": int(c.size),
                          "linked": int(lr.size), "keyed": int(h.sum())}))
    data["msg_bytes"] = np.int64(16 * world * (T.TOTAL + 4096))
    np.savez(os.path.join(work, "data.npz"), **data)
    import subprocess
    procs = [subprocess.Popen([sys.executable, "-u", os.path.join(ROOT, "tests", "_host_rank.py"),
                               ROOT, str(world), str(r), work, ",".join(scenarios)],
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
             for r in range(world)]
    for r, p in enumerate(procs):
        out, err = p.communicate(timeout=150)
        print(f"--- rank {r} rc {p.returncode}")
        print(out)
        if p.returncode:
            print(err[-3000:])


if __name__ == "__main__":
    main()
