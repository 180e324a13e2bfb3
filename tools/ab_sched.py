#!/usr/bin/env python3
"""A/B of the wave-priority rotation knob (cmpi_debug_set_sched) on the bench workloads:
back-to-back kernel timing with HIP events, both settings interleaved in one process."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bench import Workload  # noqa: E402
from cryptmpi_2022_amd import _native  # noqa: E402

modes = [int(m) for m in os.environ.get("SCHED_MODES", "0,7").split(",")]
res = {}
for wl in sys.argv[1:] or ("gcm1k", "gcm4k", "ctr1g", "ocb1m"):
    w = Workload(wl, 0, seed=3)
    times = {(m, op): [] for m in modes for op in ("seal", "open")}
    for rnd in range(6):
        for m in modes:
            _native.lib().cmpi_debug_set_sched(m)
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
                times[(m, op)].append(e0.elapsed_time(e1) / 5)
    ok = w.verify()
    for (m, op), t in times.items():
        t = sorted(t)
        res[f"{wl}_{op}_sched{m}"] = {"median_ms": round(t[len(t) // 2], 4),
                                     "GiBps": round(w.n * w.nrec / (t[len(t) // 2] * 1e-3) / 2**30, 1), "verified": ok}
    w.free()
    print(json.dumps({k: v for k, v in res.items() if k.startswith(wl)}), flush=True)
_native.lib().cmpi_debug_set_sched(7)
