#!/usr/bin/env python3
"""Per-launch durations from a rocprofv3 --kernel-trace CSV (run_kernel_trace.csv), split per
kernel and grid size (the grid tells the bench workloads apart): count, mean and median in us.
usage: rocprof_split.py <run_kernel_trace.csv> [title]"""
import collections
import csv
import sys


def main() -> None:
    path = sys.argv[1]
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0].replace("void cmpi::dev::", "")
        if "cmpi::dev" not in r["Kernel_Name"]:
            continue
        grid = r.get("Grid_Size_X") or r.get("Grid_Size") or "?"
        agg[(name, grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
    if len(sys.argv) > 2:
        print(sys.argv[2])
    for (name, grid), v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        v.sort()
        groups = [v]
        if len(v) > 20 and v[len(v) * 9 // 10] > 2.5 * v[len(v) // 10]:  # two workloads on one grid
            lo, hi = v[len(v) // 10], v[len(v) * 9 // 10]
            for _ in range(20):  # 2-means on the durations
                cut = (lo + hi) / 2
                a, b = [x for x in v if x < cut], [x for x in v if x >= cut]
                lo, hi = sum(a) / len(a), sum(b) / len(b)
            groups = [a, b]
        for gi, g in enumerate(groups):
            tag = "" if len(groups) == 1 else f" cluster {gi}"
            print(f"{name:44s} grid={grid:>8s}{tag:10s} n={len(g):6d} mean={sum(g) / len(g):9.2f} "
                  f"median={g[len(g) // 2]:9.2f}")


if __name__ == "__main__":
    main()
