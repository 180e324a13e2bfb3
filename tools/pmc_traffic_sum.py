#!/usr/bin/env python3
"""Summarise tools/pmc_traffic_ab.sh: MB per launch (FETCH_SIZE x2 gfx950 correction) per variant."""
import collections, csv, glob, json, os, sys
d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_ab"
res = {}
for var in sorted(os.listdir(d)):
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        f = glob.glob(os.path.join(d, var, c, "run_counter_collection.csv"))
        if not f:
            continue
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(f[0])):
            if "cmpi::dev" in r["Kernel_Name"]:
                agg[r["Kernel_Name"].split("(")[0].replace("void cmpi::dev::", "")].append(float(r["Counter_Value"]))
        for k, v in agg.items():
            res.setdefault(var, {}).setdefault(k, {})[c + "_MB"] = round(sum(v) / len(v) * 1024 / 1e6 * (2 if c == "FETCH_SIZE" else 1), 1)
print(json.dumps(res, indent=1))
