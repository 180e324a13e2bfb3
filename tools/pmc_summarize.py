#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (gpurun_out/pmc_<wl>/p*/run_counter_collection.csv) into
profiles/pmc_<wl>.json: per-kernel average counters and, for the dominant seal kernel, the HBM
traffic per launch corrected as MI355X_MICROARCH.md §HBM prescribes:
  FETCH_SIZE (KiB) reports 1/2 of a 16-B-per-lane streaming read on gfx950 -> x2;
  WRITE_SIZE (KiB) is exact for 16-B-per-lane streaming stores.
Only the last LAST launches of each kernel per pass are averaged (env LAST, default 0 = all): with
tools/prof_driver.py's time-based warm-up those are the sustained serial launches bench.py times.
Usage: [LAST=N] tools/pmc_summarize.py <workload> <pmc dir> <kernel substring>"""
import collections
import csv
import glob
import json
import os
import sys

wl, d, ksub = sys.argv[1], sys.argv[2], sys.argv[3]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
durs = collections.defaultdict(list)
LAST = int(os.environ.get("LAST", "0"))
for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
    rows = collections.defaultdict(list)  # kernel -> [(start, dispatch, counter, value, duration)]
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        if "cmpi::dev" not in name:
            continue
        short = name.split("(")[0].replace("void cmpi::dev::", "")
        rows[short].append((int(r["Start_Timestamp"]), r.get("Dispatch_Id", ""), r["Counter_Name"],
                            float(r["Counter_Value"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9))
    for short, rs in rows.items():
        starts = sorted({x[0] for x in rs})
        keep = set(starts[-LAST:]) if LAST else set(starts)
        seen = set()
        for st, disp, c, v, du in rs:
            if st not in keep:
                continue
            agg[short][c].append(v)
            if (st, disp) not in seen:
                seen.add((st, disp))
                durs[short].append(du)
out = {"workload": wl, "source": d, "round": os.environ.get("ROUND", "round unrecorded"), "kernels": {}}
for k, cs in agg.items():
    avg = {c: sum(v) / len(v) for c, v in cs.items()}
    dur = sum(durs[k]) / len(durs[k])
    e = {"counters_avg": {c: round(v, 1) for c, v in avg.items()}, "avg_duration_us": round(dur * 1e6, 2)}
    if "GRBM_GUI_ACTIVE" in avg:  # GPU-busy cycles summed over the XCDs, as collected (no clock derived:
        # the per-XCD division is not documented for gfx950 and gave clocks above the part's peak)
        e["grbm_gui_active"] = avg["GRBM_GUI_ACTIVE"]
    if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
        e["hbm_read_bytes"] = int(avg["FETCH_SIZE"] * 2 * 1024)
        e["hbm_write_bytes"] = int(avg["WRITE_SIZE"] * 1024)
        e["traffic_bytes_per_launch"] = e["hbm_read_bytes"] + e["hbm_write_bytes"]
    out["kernels"][k] = e
dom = [k for k in out["kernels"] if ksub in k]
if dom:
    out["dominant_kernel"] = dom[0]
    out["traffic_bytes_per_launch"] = out["kernels"][dom[0]].get("traffic_bytes_per_launch")
os.makedirs("profiles", exist_ok=True)
with open(os.path.join("profiles", f"pmc_{wl}.json"), "w") as f:
    json.dump(out, f, indent=1)
print(json.dumps({k: v.get("traffic_bytes_per_launch") for k, v in out["kernels"].items()}, indent=1))
