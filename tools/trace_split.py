"""Per-launch-shape summary of a rocprofv3 kernel trace: the bench command runs the fused
kernel for several networks and stages, so the stats CSV's one `net_kernel` average mixes
them.  Groups net_kernel dispatches by (workgroup size, grid size in threads) — one group per
config/stage — and prints count and average duration (ms) of each.

    python tools/trace_split.py gpurun_out/<tag>/trace/trace_kernel_trace.csv [OUT_CSV]
"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    groups = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if not r["Kernel_Name"].startswith("net_kernel"):
            continue
        key = (int(r["Workgroup_Size_X"]), int(r["Grid_Size_X"]))
        groups[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    rows = [("workgroup_size", "grid_size", "launches", "avg_ms", "min_ms", "max_ms")]
    for (wg, grid), ds in sorted(groups.items()):
        rows.append((wg, grid, len(ds), round(sum(ds) / len(ds), 4), round(min(ds), 4),
                     round(max(ds), 4)))
    for r in rows:
        print(",".join(str(v) for v in r))
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w", newline="") as f:
            csv.writer(f).writerows(rows)


if __name__ == "__main__":
    main()
