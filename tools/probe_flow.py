#!/usr/bin/env python3
"""Phase timeline of gcm_flow_kernel at the planner's default form (cmpi_debug_set_wide_probe):
per-workgroup wall-clock stamps (100 MHz) of start, tables staged, the first unit's Horner loop
done, its tree + chunk weight done, end — quantiles over workgroups relative to the earliest
start (us), plus the same call's host-side time per seal (HIP events over 20 calls)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# the phase probes exist only in the diagnostics build of the engine (make -C tools diag)
os.environ.setdefault("CMPI_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)), "libcmpi_aead_tools.so"))
import torch  # noqa: E402

import bench  # noqa: E402
from cryptmpi_2022_amd import _native as N  # noqa: E402

res = {}
for name, (n, nrec) in {"a2a_8x1m": (1 << 20, 8), "1x64k": (65536, 1)}.items():
    bench.WORKLOADS["_pf"] = ("gcm", n, nrec, name)
    w = bench.Workload("_pf", 0, seed=3)
    for _ in range(20):
        w.seal()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        w.seal()
    e1.record()
    torch.cuda.synchronize()
    buf = torch.zeros(8 * 4096, dtype=torch.int64, device="cuda")
    N.lib().cmpi_debug_set_wide_probe(buf.data_ptr())
    w.seal()
    torch.cuda.synchronize()
    N.lib().cmpi_debug_set_wide_probe(None)
    b = buf.view(-1, 8).cpu()
    b = b[b[:, 0] > 0]
    t0 = int(b[:, 0].min())
    q = lambda x: [round(float(v), 2) for v in torch.quantile(x, torch.tensor([0.0, 0.5, 1.0], dtype=torch.float64))]  # noqa: E731
    r = {"wgs": int(b.shape[0]), "us_per_seal_events": round(e0.elapsed_time(e1) / 20 * 1e3, 2)}
    for i, ph in [(0, "start"), (1, "staged"), (2, "horner_done"), (5, "tree_weight_done"), (6, "end")]:
        col = b[:, i]
        col = col[col > 0]
        if len(col):
            r[ph] = q((col - t0).double() / 100.0)
    end = (b[:, 6] - t0).double() / 100.0
    r["slowest_wgs"] = [int(x) for x in torch.argsort(end, descending=True)[:8]]  # rows = workgroups in order
    r["end_of_slowest"] = [round(float(end[i]), 2) for i in r["slowest_wgs"]]
    res[name] = r
    print(name, r, flush=True)
    w.free()
print(json.dumps(res))
