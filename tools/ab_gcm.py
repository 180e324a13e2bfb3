#!/usr/bin/env python3
"""Interleaved A/B timing of GCM kernel variants in ONE process (guide §5.4 rule 24):
unroll 1 vs 2 for the 1 KiB and 4 KiB configs, seal and open, median and min of N rounds."""
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
    times = {1: {"seal": [], "open": []}, 2: {"seal": [], "open": []}}
    for rnd in range(8):
        for u in (1, 2):
            N.lib().cmpi_debug_set_gcm_unroll(u)
            for op in ("seal", "open"):
                fn = w.seal if op == "seal" else w.open
                fn()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(5):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                times[u][op].append(e0.elapsed_time(e1) / 5)
    assert w.verify()
    for u in (1, 2):
        for op in ("seal", "open"):
            t = sorted(times[u][op])
            res[f"{wl}_u{u}_{op}"] = {"median_ms": round(t[len(t) // 2], 4), "min_ms": round(t[0], 4),
                                      "GiBps_median": round(w.n * w.nrec / (t[len(t) // 2] * 1e-3) / 2**30, 1)}
    w.free()
print(json.dumps(res, indent=1))
