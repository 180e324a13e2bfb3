#!/usr/bin/env python3
"""Interleaved A/B of one engine knob (a cmpi_debug_* setter taking an int) on bench workloads:
HIP-event median of seal and open per knob value, one process.

    python tools/ab_knob.py cmpi_debug_set_gcm_prefetch 2,3,4,6 gcm1k gcm4k
    python tools/ab_knob.py cmpi_debug_set_gcm_form,cmpi_debug_set_sched 1:7,0:16391 gcm1k   (several knobs)
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bench import Workload  # noqa: E402
from cryptmpi_2022_amd import _native as N  # noqa: E402

_setters = [getattr(N.lib(), n) for n in sys.argv[1].split(",")]
values = sys.argv[2].split(",")


def setter(v):
    for fn, x in zip(_setters, str(v).split(":")):
        fn(int(x))
res = {}
for wl in sys.argv[3:]:
    w = Workload(wl, 0, seed=3)
    t = {(v, op): [] for v in values for op in ("seal", "open")}
    alt = os.environ.get("ABK_ALT") == "1"  # bench.py's timing: seal/open alternating per step
    for rnd in range(int(os.environ.get("ABK_ROUNDS", "7"))):
        for v in values:
            setter(v)
            if alt:
                w.seal()
                w.open()
                torch.cuda.synchronize()
                ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(4)]
                for e0, e1, e2 in ev:
                    e0.record()
                    w.seal()
                    e1.record()
                    w.open()
                    e2.record()
                torch.cuda.synchronize()
                t[(v, "seal")].append(sum(a.elapsed_time(b) for a, b, _ in ev) / 4)
                t[(v, "open")].append(sum(b.elapsed_time(c) for _, b, c in ev) / 4)
                continue
            for op in ("seal", "open"):
                fn = w.seal if op == "seal" else w.open
                fn()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(4):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                t[(v, op)].append(e0.elapsed_time(e1) / 4)
    ok = w.verify()
    for (v, op), ts in t.items():
        m = sorted(ts)[len(ts) // 2]
        res[f"{wl}_{op}_{v}"] = {"ms": round(m, 4), "GiBps": round(w.n * w.nrec / (m * 1e-3) / 2**30, 1)}
    res[f"{wl}_verified"] = ok
    setter(values[0])
    w.free()
print(json.dumps(res, indent=0))
