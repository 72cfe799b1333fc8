#!/usr/bin/env python3
"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes into per-kernel HBM bytes
per launch (profiles/<round>/pmc_traffic.json, read by bench.py's roofline).

Units and gfx950 corrections follow /opt/skills/guides/MI355X_MICROARCH.md
(HBM section): both counters are in KiB; FETCH_SIZE of wide (16 B/lane)
streaming reads is exactly half the bytes on gfx950, so it is doubled;
WRITE_SIZE is exact for 16-B-per-lane stores.

Usage: python scripts/pmc_summary.py <prof_dir> <out.json> [kernel-substring ...]
"""
import collections
import csv
import json
import os
import re
import sys


def kernel_key(name: str) -> str:
    """k_<name>, plus ':ListOut' for the group kernels' list-output variant
    (round 4: the RepOut / ListOut instantiations are separate kernels)."""
    m = re.search(r"(k_\w+)", name)
    k = m.group(1) if m else name[:80]
    return k + ":ListOut" if "ListOut" in name else k


def load(path, counter):
    agg = collections.defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] != counter:
                continue
            agg[kernel_key(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return agg


def main():
    prof, out = sys.argv[1], sys.argv[2]
    want = sys.argv[3:]
    fetch = load(os.path.join(prof, "pmc_FETCH_SIZE", "pmc_counter_collection.csv"), "FETCH_SIZE")
    write = load(os.path.join(prof, "pmc_WRITE_SIZE", "pmc_counter_collection.csv"), "WRITE_SIZE")
    res = {}
    for k in sorted(set(fetch) | set(write)):
        if want and not any(w in k for w in want):
            continue
        f = fetch.get(k, [])
        w = write.get(k, [])
        fb = 2 * 1024 * sum(f) / len(f) if f else None
        wb = 1024 * sum(w) / len(w) if w else None
        res[k] = {"fetch_bytes_per_launch": fb, "write_bytes_per_launch": wb,
                  "hbm_bytes_per_launch": (fb or 0) + (wb or 0), "launches": max(len(f), len(w))}
    # effective clock per kernel (MI355X_MICROARCH.md 'DVFS give-back'):
    # GRBM_GUI_ACTIVE summed over the 8 XCDs / 8 / dispatch wall time
    clk = {}
    gpath = os.path.join(prof, "pmc_GRBM_GUI_ACTIVE_GRBM_COUNT", "pmc_counter_collection.csv")
    if os.path.exists(gpath):
        acc = collections.defaultdict(list)
        with open(gpath) as f:
            for r in csv.DictReader(f):
                if r["Counter_Name"] != "GRBM_GUI_ACTIVE":
                    continue
                k = kernel_key(r["Kernel_Name"])
                dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
                if dur > 0:
                    acc[k].append(float(r["Counter_Value"]) / 8 / dur / 1e9)
        clk = {k: sum(v) / len(v) for k, v in acc.items()}
        for k, v in res.items():
            if k in clk:
                v["effective_clock_GHz"] = clk[k]
    doc = {"source": prof, "correction": "FETCH_SIZE KiB x 1024 x 2 (gfx950 half-count of "
           "16-B/lane streaming reads), WRITE_SIZE KiB x 1024", "kernels": res}
    with open(out, "w") as fo:
        json.dump(doc, fo, indent=1)
    for k, v in res.items():
        print(f"{k:32s} fetch {v['fetch_bytes_per_launch'] or 0:.4g} B  write "
              f"{v['write_bytes_per_launch'] or 0:.4g} B  clock "
              f"{v.get('effective_clock_GHz', 0):.3f} GHz")


if __name__ == "__main__":
    main()
