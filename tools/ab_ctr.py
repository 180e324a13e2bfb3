#!/usr/bin/env python3
"""Occupancy experiment on the pure-AES CTR kernel (one process, interleaved rounds): LDS
request 64 KiB (2 blocks/CU = 8 waves/SIMD) vs 96 KiB (1 block/CU = 4 waves/SIMD)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bench import Workload  # noqa: E402
from cryptmpi_2022_amd import _native as N  # noqa: E402

w = Workload("ctr1g", 0, seed=3)
variants = [65536, 98304]
t = {v: [] for v in variants}
for rnd in range(6):
    for v in variants:
        N.lib().cmpi_debug_set_ctr_lds(v)
        w.seal()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            w.seal()
        e1.record()
        torch.cuda.synchronize()
        t[v].append(e0.elapsed_time(e1) / 3)
N.lib().cmpi_debug_set_ctr_lds(65536)
res = {}
for v, ts in t.items():
    ts.sort()
    res[f"lds{v // 1024}K"] = {"median_ms": round(ts[len(ts) // 2], 3),
                                               "GiBps": round(w.n / (ts[len(ts) // 2] * 1e-3) / 2**30, 1)}
print(json.dumps(res, indent=1))
