#!/usr/bin/env python3
"""Back-to-back kernel timing (HIP events, median/min of rounds, one process) of seal and open
for the bench workloads — the per-kernel view next to bench.py's end-to-end step timing."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bench import Workload  # noqa: E402

res = {}
for wl in sys.argv[1:] or ("gcm1k", "gcm4k", "ctr1g", "ocb1m"):
    w = Workload(wl, 0, seed=3)
    times = {"seal": [], "open": []}
    for rnd in range(8):
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
            times[op].append(e0.elapsed_time(e1) / 5)
    ok = w.verify()
    for op in ("seal", "open"):
        t = sorted(times[op])
        res[f"{wl}_{op}"] = {"median_ms": round(t[len(t) // 2], 4), "min_ms": round(t[0], 4),
                             "GiBps_median": round(w.n * w.nrec / (t[len(t) // 2] * 1e-3) / 2**30, 1), "verified": ok}
    w.free()
print(json.dumps(res, indent=1))
