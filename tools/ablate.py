#!/usr/bin/env python3
"""Timing ablation of the GCM seal kernel, interleaved rounds in one process (results of
ablated runs are wrong by construction).  Modes: full / no GHASH / no AES / neither, each with
record addressing and with a coalesced stand-in stream, for forced lanes-per-record L."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bench import Workload  # noqa: E402
from cryptmpi_2022_amd import _native as N  # noqa: E402
from cryptmpi_2022_amd import aead  # noqa: E402

MODES = {0: "full", 1: "noghash", 2: "noaes", 3: "neither", 4: "full_coal", 7: "neither_coal"}
res = {}
for wl in ("gcm1k", "gcm4k"):
    w = Workload(wl, 0, seed=3)
    for L in (4, 2, 1):
        aead.force_plan(L, 0)
        t = {m: [] for m in MODES}
        for rnd in range(5):
            for m in MODES:
                N.lib().cmpi_debug_set_gcm_ablation(m)
                w.seal()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(4):
                    w.seal()
                e1.record()
                torch.cuda.synchronize()
                t[m].append(e0.elapsed_time(e1) / 4)
        for m, ts in t.items():
            ts.sort()
            res[f"{wl}_L{L}_{MODES[m]}"] = round(ts[len(ts) // 2], 4)
    N.lib().cmpi_debug_set_gcm_ablation(0)
    aead.force_plan(0, 0)
    w.free()
print(json.dumps(res, indent=1))
