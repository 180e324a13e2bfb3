#!/usr/bin/env python3
"""Minimal driver for rocprofv3 (kernel-trace / PMC passes): runs `iters` seal+open steps of one
bench workload on cuda:0, nothing else (no distributed init, no CPU baseline)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from bench import Workload  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="gcm1k")
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--seal-only", action="store_true")
a = ap.parse_args()
w = Workload(a.workload, 0, seed=1)
for _ in range(a.iters):
    w.seal()
    if not a.seal_only:
        w.open()
torch.cuda.synchronize()
print("ok", a.workload, w.verify() if not a.seal_only else "seal-only")
