#!/usr/bin/env python3
"""Timing ablation of the GCM seal kernel (L = 4 plan): full / no GHASH / no AES / neither,
interleaved rounds in one process.  Results of ablated runs are wrong by construction."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bench import Workload  # noqa: E402
from cryptmpi_2022_amd import _native as N  # noqa: E402

res = {}
for wl in ("gcm1k", "gcm4k"):
    w = Workload(wl, 0, seed=3)
    t = {m: [] for m in range(4)}
    for rnd in range(6):
        for m in range(4):
            N.lib().cmpi_debug_set_gcm_ablation(m)
            w.seal()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                w.seal()
            e1.record()
            torch.cuda.synchronize()
            t[m].append(e0.elapsed_time(e1) / 5)
    N.lib().cmpi_debug_set_gcm_ablation(0)
    for m, ts in t.items():
        ts.sort()
        res[f"{wl}_{['full', 'noghash', 'noaes', 'neither'][m]}"] = round(ts[len(ts) // 2], 4)
    w.free()
print(json.dumps(res, indent=1))
