"""Per-workload kernel averages from a rocprofv3 kernel trace.

rocprofv3 --stats averages every launch of a kernel, and the bench launches
the same kernels at several sizes (the 1 M-file headline step, the config-1
directory, single-file latency, 12.5 M-row dedup, 1 M-row job grouping).
This splits launches by grid size and, for the persistent K1 grid (constant
grid), by duration, so the average for the headline workload can be compared
with the HIP-event average bench.py reports.

usage: python scripts/trace_summary.py <run_kernel_trace.csv> [out.txt]
"""
import collections
import csv
import sys

# first match wins: the longer names before their prefixes
KERNELS = ["k_leaves3", "k_fold3", "k_tree_level<true>", "k_tree_level<false>",
           "k_part_hist", "k_part_scatter_runs", "k_part_scatter_rec_staged", "k_part_scatter_rec",
           "k_part_scatter_ws", "k_part_private", "k_part2_runs", "k_fine_recount_runs",
           "k_fine_scan", "k_bucket_group12_pk", "k_bucket_group_pk",
           "k_bucket_group12", "k_bucket_group", "k_window_apply", "k_link_count", "k_link_write",
           "k_keyless_count", "k_keyless_write", "k_ret_count", "k_ret_write", "k_ret_apply",
           "k_gather_rep", "k_small_host", "k_small_split", "k_service"]
LONG_MS = 5.0  # K1 launches over a whole 1 M-file step take ~13 ms; every other K1 launch < 2 ms


def main(path, out=None):
    groups = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        short = next((k for k in KERNELS if k in name), None)
        if short is None:
            continue
        if "ListOut" in name:  # the group kernels' list-output instantiation (round 4)
            short += ":ListOut"
        ms = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        key = (short, int(r["Grid_Size_X"]))
        if short in ("k_leaves3", "k_fold3"):
            key = (short, "1M-file step" if ms >= LONG_MS or short == "k_fold3" and ms > 0.1
                   else "other")
        groups[key].append(ms)
    lines = [f"{'kernel':26s} {'group':>14s} {'launches':>8s} {'avg_ms':>10s} {'median_ms':>10s} "
             f"{'min_ms':>9s} {'max_ms':>9s}"]
    for (k, g), v in sorted(groups.items(), key=lambda kv: (kv[0][0], str(kv[0][1]))):
        med = sorted(v)[len(v) // 2]
        lines.append(f"{k:26s} {str(g):>14s} {len(v):8d} {sum(v) / len(v):10.4f} {med:10.4f} "
                     f"{min(v):9.4f} {max(v):9.4f}")
    text = "\n".join(lines)
    print(text)
    if out:
        open(out, "w").write(text + "\n")


if __name__ == "__main__":
    main(*sys.argv[1:])
