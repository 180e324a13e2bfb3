#!/usr/bin/env python3
"""FLOW wide GCM kernel variants on few long records (BASELINE config 5 per rank: 8 x 1 MiB;
also 64 x 1 MiB and 1 x 64 KiB): round-1 gcm_wide_kernel + combine vs gcm_flow_kernel at 512 /
1024 threads per workgroup, combine fused or not, steps per chunk.  Seal/open time per call from
back-to-back launches (torch events over 5 calls, median of 6 rounds); every variant's output is
checked (round trip + oracle tags of the first 2 records)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import oracle  # noqa: E402
from cryptmpi_2022_amd import _native as N  # noqa: E402
from cryptmpi_2022_amd import aead  # noqa: E402

SHAPES = {"a2a_8x1m": (1 << 20, 8), "64x1m": (1 << 20, 64), "1x64k": (65536, 1)}
VARIANTS = [("r1", 0, 1), ("flow1024_unfused", 1024, 0), ("flow1024", 1024, 1), ("flow512", 512, 1),
            ("w4_1024_unfused", 1024, 16), ("w4_1024", 1024, 17), ("fixed1024", 1024, 32), ("fixed512", 512, 32)]
# timing ablations (output wrong, not verified), fused: skip tree (2), chunk-weight product (4), AES (8)
VARIANTS += [(f"abl{c}", 1024, c | 1) for c in (2, 4, 6, 8, 14)]
# unfused ablations incl. no stores (128) / no loads (256)
VARIANTS += [(f"ablu{c}", 1024, c) for c in (2, 4, 8, 14, 128, 256, 384, 398)]
only = sys.argv[1:]
res = {}
for name, (n, nrec) in SHAPES.items():
    bench.WORKLOADS["_ab"] = ("gcm", n, nrec, name)
    for vname, nt, fused in VARIANTS:
        for steps in [int(x) for x in os.environ.get("AB_STEPS", "0,1,2,4,8").split(",")]:
            if only and f"{name}:{vname}" not in only and name not in only:
                continue
            N.lib().cmpi_debug_set_flow(nt, fused)
            aead.force_wide(1, steps)
            w = bench.Workload("_ab", 0, seed=3)
            plan = aead.gcm_plan(w.ctx, n, nrec)
            times = {"seal": [], "open": []}
            for _ in range(6):
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
            if fused & (14 | 128 | 256):
                res[f"{name}:{vname}:S{steps or 'auto'}"] = {op: round(sorted(t)[3] * 1e3, 1) for op, t in times.items()}
                print(name, vname, steps, res[f"{name}:{vname}:S{steps or 'auto'}"], flush=True)
                w.free()
                continue
            ok = w.verify()
            k = min(2, nrec)
            pt = w.pt[: k * n].cpu().numpy().reshape(k, n)
            nn = w.nonces[: k * 12].cpu().numpy().reshape(k, 12)
            ct = w.ct[: k * (n + 16)].cpu().numpy().reshape(k, n + 16)
            ok = ok and np.array_equal(ct, oracle.gcm_seal_batch(bytes(range(16)), nn, pt))
            key = f"{name}:{vname}:S{steps or 'auto'}"
            res[key] = {"plan": plan, "verified": bool(ok)}
            for op in ("seal", "open"):
                t = sorted(times[op])[len(times[op]) // 2]
                res[key][f"{op}_us"] = round(t * 1e3, 1)
                res[key][f"{op}_GiBps"] = round(n * nrec / (t * 1e-3) / 2**30, 1)
            w.free()
            print(key, res[key], flush=True)
N.lib().cmpi_debug_set_flow(1024, 0)
aead.force_wide(0, 0)
print(json.dumps(res))
