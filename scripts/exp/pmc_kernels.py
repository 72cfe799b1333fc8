"""Per-kernel averages of rocprofv3 --pmc counter CSVs under a directory
(one line per kernel name and counter set), for the grouping kernels.

    python scripts/exp/pmc_kernels.py <dir>
"""
import collections
import csv
import glob
import os
import re
import sys

KEEP = ("k_part_private", "k_part2_runs", "k_fine_scan", "k_bucket_group12_pk", "k_bucket_group12_glds",
        "k_bucket_group_pk", "k_part_hist", "k_part_scatter_ws", "k_list_finish")


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"^void ", "", name)
    name = re.sub(r"\(.*", "", name)
    for k in KEEP:
        if k in name:
            return k + (":ListOut" if "ListOut" in name else "")
    return None


def main(root):
    for sub in sorted(os.listdir(root)):
        files = glob.glob(os.path.join(root, sub, "**", "*counter_collection.csv"), recursive=True)
        if not files:
            continue
        acc = collections.defaultdict(lambda: collections.defaultdict(list))
        for f in files:
            for r in csv.DictReader(open(f)):
                k = short(r.get("Kernel_Name", ""))
                if not k:
                    continue
                grid = r.get("Grid_Size", r.get("Grid_Size_X", ""))
                acc[(k, grid)][r["Counter_Name"]].append(float(r["Counter_Value"]))
        print(f"== {sub}")
        for (k, grid), cs in sorted(acc.items()):
            vals = {c: sum(v) / len(v) for c, v in cs.items()}
            print(f"  {k} grid={grid} " + " ".join(f"{c}={v:.4g}" for c, v in sorted(vals.items())))


if __name__ == "__main__":
    main(sys.argv[1])
