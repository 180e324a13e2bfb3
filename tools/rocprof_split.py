#!/usr/bin/env python3
"""Per-launch durations from a rocprofv3 --kernel-trace CSV (run_kernel_trace.csv), split per
kernel, grid size and schedule phase: count, mean and median in us.

A phase is a run of launches of one (kernel, grid) with no gap longer than --gap-ms between two
consecutive launches.  bench.py separates its workloads by CPU-side parity checks that take far
longer than that, so each phase is one workload's pass (the headline's untimed first step, its
warm-up + timed steps, the gcm4k extra, ...), told apart by when they ran rather than by how long
each launch took.  Phases shorter than --min-n launches are folded into one "other" line.

usage: rocprof_split.py <run_kernel_trace.csv> [title] [--gap-ms 20] [--min-n 50]"""
import argparse
import collections
import csv


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("title", nargs="?")
    ap.add_argument("--gap-ms", type=float, default=20.0)
    ap.add_argument("--min-n", type=int, default=50)
    a = ap.parse_args()
    launches = collections.defaultdict(list)  # (name, grid) -> [(start_ns, dur_us)]
    for r in csv.DictReader(open(a.csv)):
        if "cmpi::dev" not in r["Kernel_Name"]:
            continue
        name = r["Kernel_Name"].split("(")[0].replace("void cmpi::dev::", "")
        grid = r.get("Grid_Size_X") or r.get("Grid_Size") or "?"
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        launches[(name, grid)].append((s, (e - s) * 1e-3))
    if a.title:
        print(a.title)
    gap = a.gap_ms * 1e6
    for (name, grid), v in sorted(launches.items(), key=lambda kv: -sum(d for _, d in kv[1])):
        v.sort()
        phases, cur = [], [v[0]]
        for prev, x in zip(v, v[1:]):
            if x[0] - prev[0] > gap:
                phases.append(cur)
                cur = []
            cur.append(x)
        phases.append(cur)
        big = [p for p in phases if len(p) >= a.min_n]
        small = [x for p in phases if len(p) < a.min_n for x in p]
        rows = [(f"phase {i}", p) for i, p in enumerate(big)] + ([("other", small)] if small else [])
        t0 = v[0][0]
        for tag, p in rows:
            d = sorted(x for _, x in p)
            when = "" if tag == "other" else f" t={(p[0][0] - t0) * 1e-9:7.3f}s"
            print(f"{name:44s} grid={grid:>8s} {tag:8s}{when:11s} n={len(d):6d} mean={sum(d) / len(d):9.2f} "
                  f"median={d[len(d) // 2]:9.2f}")


if __name__ == "__main__":
    main()
