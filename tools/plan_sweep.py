#!/usr/bin/env python3
"""GCM seal time (device-resident, back-to-back median) under the automatic plan vs forced wide
S=1 vs forced lane groups, for batches between single messages and a full chip."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from cryptmpi_2022_amd import aead  # noqa: E402

key = bytes(range(16))
ctx = aead.AeadCtx(key)
cases = [(1024, 1), (1024, 64), (1024, 1024), (1024, 4096), (1024, 16384), (1024, 32768),
         (2048, 4096), (4096, 4096), (16384, 256), (16384, 4096)]
for n, nrec in cases:
    pt = torch.randint(0, 256, (n * nrec,), dtype=torch.uint8, device="cuda")
    nn = torch.randint(0, 256, (12 * nrec,), dtype=torch.uint8, device="cuda")
    out = torch.empty((n + 16) * nrec, dtype=torch.uint8, device="cuda")
    row = {}
    for name, fw in (("auto", (0, 0)), ("wideS1", (1, 1)), ("wideS2", (1, 2)), ("lanes", (-1, 0))):
        aead.force_wide(*fw)
        plan = aead.gcm_plan(ctx, n, nrec)
        ws = torch.empty(max(16, ctx.workspace_size(n, nrec)), dtype=torch.uint8, device="cuda")
        ctx.seal_batch(out, pt, nn, n, nrec, workspace=ws)
        torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                ctx.seal_batch(out, pt, nn, n, nrec, workspace=ws)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / 10 * 1e3)
        ts.sort()
        row[name] = (round(ts[2], 1), list(plan))
    aead.force_wide(0, 0)
    print(n, nrec, json.dumps(row), flush=True)
