#!/usr/bin/env python3
"""Gap between consecutive config-2 seal launches on one stream, for the rocprofv3 kernel trace:
phase A launches 40 seals back to back, phase B 40 seals with a fence-free event (the bench's
KernelEvents) after each, phase C 40 seals with a default torch event after each.  Run under
`rocprofv3 --kernel-trace` and read the gaps with tools/rocpd_summary.py or the CSV trace."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

w = bench.Workload("gcm1k", 0, seed=3)
for _ in range(20):
    w.seal()
torch.cuda.synchronize()
stream = torch.cuda.current_stream().cuda_stream
for _ in range(40):
    w.seal()
torch.cuda.synchronize()
ev = bench.KernelEvents(41)
for i in range(40):
    w.seal()
    ev.record(i, stream)
torch.cuda.synchronize()
tev = [torch.cuda.Event(enable_timing=True) for _ in range(40)]
for i in range(40):
    w.seal()
    tev[i].record()
torch.cuda.synchronize()
ev.free()
print("gap_probe done")
