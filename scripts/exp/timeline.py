"""Kernel timeline of a rocprofv3 kernel trace: the last N kernels in start
order with their durations and the idle gap before each, and per-name totals.

    python scripts/exp/timeline.py <run_kernel_trace.csv> [N] [skip_last]
"""
import collections
import csv
import re
import sys


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"^void ", "", name)
    name = re.sub(r"\(.*", "", name)
    return name[:70]


def main(path, n=80, skip_last=0):
    rs = []
    for r in csv.DictReader(open(path)):
        rs.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                   int(r["Grid_Size_X"])))
    rs.sort()
    if skip_last:
        rs = rs[:-skip_last]
    sel = rs[-n:]
    prev_end = None
    busy = 0
    for s, e, k, g in sel:
        gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
        print(f"{gap:9.1f} us gap  {(e - s) / 1e3:9.1f} us  grid {g:9d}  {k}")
        prev_end = max(prev_end or 0, e)
        busy += e - s
    span = (sel[-1][1] - sel[0][0]) / 1e3
    print(f"span {span:.1f} us, busy {busy / 1e3:.1f} us")
    tot = collections.defaultdict(float)
    for s, e, k, g in sel:
        tot[k] += (e - s) / 1e3
    for k, v in sorted(tot.items(), key=lambda x: -x[1]):
        print(f"{v:10.1f} us  {k}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 80,
         int(sys.argv[3]) if len(sys.argv) > 3 else 0)
