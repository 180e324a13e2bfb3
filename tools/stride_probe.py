#!/usr/bin/env python3
"""Does the record stride (power of two vs padded) change GCM seal time?  One process,
interleaved rounds; plus the 'neither' ablation (memory path only)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from cryptmpi_2022_amd import _native as N  # noqa: E402
from cryptmpi_2022_amd import aead  # noqa: E402

res = {}
ctx = aead.AeadCtx(bytes(range(16)))
for n, N_ in ((1024, 65536), (4096, 65536)):
    for pad in (0, 64, 256, 16):
        ins, outs = n + pad, n + 16 + pad
        pt = torch.randint(0, 256, (N_ * ins,), dtype=torch.uint8, device="cuda")
        nn = torch.randint(0, 256, (N_ * 12,), dtype=torch.uint8, device="cuda")
        ct = torch.empty(N_ * outs, dtype=torch.uint8, device="cuda")
        for m in (0, 3):
            N.lib().cmpi_debug_set_gcm_ablation(m)
            ts = []
            for rnd in range(5):
                ctx.seal_batch(ct, pt, nn, n, N_, in_stride=ins, out_stride=outs)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(4):
                    ctx.seal_batch(ct, pt, nn, n, N_, in_stride=ins, out_stride=outs)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) / 4)
            ts.sort()
            res[f"n{n}_pad{pad}_{'full' if m == 0 else 'neither'}"] = round(ts[2], 4)
        del pt, ct, nn
N.lib().cmpi_debug_set_gcm_ablation(0)
print(json.dumps(res, indent=1))
