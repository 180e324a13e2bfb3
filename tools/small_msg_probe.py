#!/usr/bin/env python3
"""Single-message latency of the GCM seal (device-resident, back-to-back median) by plan: automatic,
wide with forced steps per chunk, lane groups with forced segments — the config-1 / drop-in regime."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from cryptmpi_2022_amd import aead  # noqa: E402

key = bytes(range(16))
res = {}
for n in (4096, 16384, 65536, 1 << 20):
    ctx = aead.AeadCtx(key)
    pt = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda")
    nn = torch.randint(0, 256, (12,), dtype=torch.uint8, device="cuda")
    out = torch.empty(n + 16, dtype=torch.uint8, device="cuda")
    ws = torch.empty(max(16, 1 << 20), dtype=torch.uint8, device="cuda")
    variants = [("auto", lambda: (aead.force_wide(0, 0), aead.force_plan(0, 0)))]
    for S in (1, 2, 4, 8):
        variants.append((f"wide_S{S}", lambda S=S: (aead.force_wide(1, S), aead.force_plan(0, 0))))
    for seg in (8, 32, 128):
        variants.append((f"lanes4_seg{seg}", lambda seg=seg: (aead.force_wide(-1, 0), aead.force_plan(4, seg))))
    row = {}
    for name, setup in variants:
        setup()
        try:
            plan = aead.gcm_plan(ctx, n, 1)
            ctx.seal_batch(out, pt, nn, n, 1, workspace=ws)
            torch.cuda.synchronize()
            ts = []
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(20):
                    ctx.seal_batch(out, pt, nn, n, 1, workspace=ws)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) / 20 * 1e3)
            ts.sort()
            row[name] = {"us": round(ts[2], 1), "plan": list(plan)}
        except Exception as e:
            row[name] = {"error": repr(e)[:80]}
    aead.force_wide(0, 0)
    aead.force_plan(0, 0)
    res[n] = row
    print(n, json.dumps(row), flush=True)
    ctx.close()
