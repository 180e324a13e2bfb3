#!/usr/bin/env python3
"""Per-kernel duration summary (count, median, mean, min in us) from a rocprofv3 results.db
(--kernel-trace), optionally only kernels whose name contains a filter string."""
import collections
import sqlite3
import sys


def summary(db: str, filt: str = "") -> dict:
    c = sqlite3.connect(db)
    names = [r[0] for r in c.execute("select name from sqlite_master where type='table'")]
    suf = [n for n in names if n.startswith("rocpd_kernel_dispatch")][0].split("dispatch_")[1]
    q = (f"select s.kernel_name, d.start, d.end from rocpd_kernel_dispatch_{suf} d "
         f"join rocpd_info_kernel_symbol_{suf} s on d.kernel_id = s.id order by d.start")
    agg = collections.defaultdict(list)
    for n, s, e in c.execute(q):
        if filt in n:
            agg[n].append((e - s) / 1000.0)
    out = {}
    for n, v in agg.items():
        v.sort()
        out[n] = {"count": len(v), "median_us": round(v[len(v) // 2], 2), "mean_us": round(sum(v) / len(v), 2),
                  "min_us": round(v[0], 2)}
    return out


if __name__ == "__main__":
    for n, r in summary(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "").items():
        print(f"{r['count']:6d} med {r['median_us']:9.2f} mean {r['mean_us']:9.2f} min {r['min_us']:9.2f}  {n[:110]}")
