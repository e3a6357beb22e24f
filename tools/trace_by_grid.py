"""Per-(kernel, grid size) summary of a rocprofv3 --kernel-trace CSV.

bench.py runs the same kernels at several sizes (configs[1] TPKE, configs[2] CommonCoin, configs[4] epoch
replay), so the per-kernel averages of --stats mix workloads; grouping by grid size separates them.
Usage: python tools/trace_by_grid.py <run_kernel_trace.csv>
"""
import collections
import csv
import sys


def main(path):
    groups = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        groups[(r["Kernel_Name"], int(r["Grid_Size_X"]))].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    print(f"{'kernel':40s} {'grid_lanes':>10s} {'calls':>5s} {'avg_ms':>10s} {'total_ms':>10s}")
    for (name, grid), d in sorted(groups.items(), key=lambda kv: -sum(kv[1])):
        if sum(d) < 1e6:
            continue
        print(f"{name[:40]:40s} {grid:10d} {len(d):5d} {sum(d) / len(d) / 1e6:10.2f} {sum(d) / 1e6:10.1f}")


if __name__ == "__main__":
    main(sys.argv[1])
