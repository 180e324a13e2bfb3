#!/usr/bin/env python3
"""Wide vs lane-group GCM decomposition on few long records (BASELINE config 5 per rank:
8 x 1 MiB, plus 64 x 1 MiB and 4096 x 1 MiB): seal/open kernel time (HIP events, median of
rounds) for the lane-group plan and the wide plan at several steps-per-chunk."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from cryptmpi_2022_amd import aead  # noqa: E402

SHAPES = {"alltoall": (1 << 20, 8), "gcm64x1m": (1 << 20, 64), "gcm4096x1m": (1 << 20, 4096)}
res = {}
for name, (n, nrec) in SHAPES.items():
    bench.WORKLOADS["_ab"] = ("gcm", n, nrec, name)
    for mode, steps in [(-1, 0)] + [(1, s) for s in (1, 2, 4, 8, 16, 0)]:
        if nrec >= 4096 and steps in (1, 2):
            continue
        aead.force_wide(mode, steps)
        w = bench.Workload("_ab", 0, seed=3)
        plan = aead.gcm_plan(w.ctx, n, nrec)
        times = {"seal": [], "open": []}
        for rnd in range(6):
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
        key = f"{name}_{'lanes' if mode < 0 else 'wide_S' + str(steps or 'auto')}"
        res[key] = {"plan": plan, "verified": ok}
        for op in ("seal", "open"):
            t = sorted(times[op])[len(times[op]) // 2]
            res[key][f"{op}_us"] = round(t * 1e3, 1)
            res[key][f"{op}_GiBps"] = round(n * nrec / (t * 1e-3) / 2**30, 1)
        w.free()
        print(key, res[key], flush=True)
aead.force_wide(0, 0)
print(json.dumps(res))
