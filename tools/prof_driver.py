#!/usr/bin/env python3
"""Minimal driver for rocprofv3 (kernel-trace / PMC passes): runs `iters` seal+open steps of one
bench workload on cuda:0, nothing else (no distributed init, no CPU baseline).  The steps follow
--warmup-s seconds of untimed steps (default 0.5, as bench.py's headline), so that the last
`iters` launches of each kernel are the sustained, serial ones bench.py times; summarise only those
(tools/pmc_summarize.py LAST=<iters>, tools/rocprof_split.py --last <iters>)."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from bench import Workload  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="gcm1k")
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--seal-only", action="store_true")
ap.add_argument("--warmup-s", type=float, default=0.5)
ap.add_argument("--out-stride", type=int, default=0,
                help="gcm1k seal-only traffic calibration: output record stride (0 = dense n+16)")
a = ap.parse_args()
for kv in filter(None, os.environ.get("AB_HOOKS", "").split(",")):  # test hooks, e.g. lane_aligned=0
    from cryptmpi_2022_amd import _native as _N

    k, v = kv.split("=")
    getattr(_N.lib(), "cmpi_debug_set_" + k)(int(v))
if a.out_stride:  # 65 536 x 1 KiB seals into records `out_stride` bytes apart (aligned vs dense)
    from cryptmpi_2022_amd import aead

    n, nrec = 1024, 65536
    ctx = aead.AeadCtx(bytes(range(16)))
    pt = torch.randint(0, 256, (nrec * n,), dtype=torch.uint8, device="cuda")
    nn = torch.randint(0, 256, (nrec * 12,), dtype=torch.uint8, device="cuda")
    out = torch.empty(nrec * a.out_stride, dtype=torch.uint8, device="cuda")
    for _ in range(a.iters):
        ctx.seal_batch(out, pt, nn, n, nrec, out_stride=a.out_stride)
    torch.cuda.synchronize()
    print("ok out_stride", a.out_stride)
    sys.exit(0)
w = Workload(a.workload, 0, seed=1)
t_end = time.perf_counter() + a.warmup_s
while time.perf_counter() < t_end:
    for _ in range(10):
        w.seal()
        if not a.seal_only:
            w.open()
    torch.cuda.synchronize()
for _ in range(a.iters):
    w.seal()
    if not a.seal_only:
        w.open()
torch.cuda.synchronize()
print("ok", a.workload, w.verify() if not a.seal_only else "seal-only")
