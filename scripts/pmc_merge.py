#!/usr/bin/env python3
"""Merge the per-workload PMC summaries of scripts/gpu_r3_profile.sh
(gpu_r4/r5/r6_profile.sh: pmc_cas.json, pmc_dedup.json, pmc_dedup_full.json, each written by
scripts/pmc_summary.py) into the one file bench.py reads:
profiles/<round>/pmc_traffic.json with sections "kernels" (config-2 K1 step),
"dedup" (12.5 M-row grouping) and "dedup_full" (100 M-row two-level grouping).

Usage: python scripts/pmc_merge.py <prof_dir> <out.json> <tag>
"""
import json
import os
import sys


def main():
    prof, out, tag = sys.argv[1], sys.argv[2], sys.argv[3]
    doc = {"source": f"rocprofv3 --pmc passes of the round's scripts/gpu_r<round>_profile.sh (TAG={tag}): "
                     "'kernels' = bench.py --components cas (config-2 1M-file step), "
                     "'dedup' = bench.py --components dedup --dedup-full-rows 0 (12.5M-row "
                     "grouping), 'dedup_full' = --dedup-rows 100000000 --dedup-full-rows 0 "
                     "(100M-row two-level grouping)"}
    for sec, name in (("kernels", "pmc_cas.json"), ("dedup", "pmc_dedup.json"),
                      ("dedup_full", "pmc_dedup_full.json")):
        p = os.path.join(prof, name)
        if not os.path.exists(p):
            continue
        d = json.load(open(p))
        doc.setdefault("correction", d.get("correction"))
        doc[sec] = d["kernels"]
    with open(out, "w") as fo:
        json.dump(doc, fo, indent=1)


if __name__ == "__main__":
    main()
