#!/usr/bin/env python3
"""Timeline of the GCM lane-group kernel (cmpi_debug_set_wide_probe also arms it): per workgroup
its start, tables-staged and the end of waves 0..5 (100 MHz wall clock), relative to the earliest
start — to see dispatch skew, staging cost and how far apart equal-work waves finish."""
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
for wl in (sys.argv[1:] or ["gcm1k", "gcm4k"]):
    w = bench.Workload(wl, 0, seed=3)
    buf = torch.zeros(8 * 4096, dtype=torch.int64, device="cuda")
    for _ in range(20):
        w.seal()
    torch.cuda.synchronize()
    N.lib().cmpi_debug_set_wide_probe(buf.data_ptr())
    w.seal()
    torch.cuda.synchronize()
    N.lib().cmpi_debug_set_wide_probe(None)
    b = buf.view(-1, 8).cpu()
    b = b[b[:, 0] > 0]
    t0 = int(b[:, 0].min())
    rel = (b - t0).double() / 100.0  # us
    q = lambda x: [round(float(v), 2) for v in torch.quantile(x, torch.tensor([0.0, 0.5, 1.0], dtype=torch.float64))]  # noqa: E731
    ends = rel[:, 2:8].reshape(-1)
    spread = (rel[:, 2:8].max(dim=1).values - rel[:, 2:8].min(dim=1).values)
    idx = torch.nonzero(buf.view(-1, 8)[:, 0].cpu() > 0).view(-1)
    wg_end = rel[:, 2:8].max(dim=1).values
    by_xcd = {int(x): round(float(wg_end[(idx % 8) == x].median()), 2) for x in range(8)}
    res[wl] = {"wgs": int(b.shape[0]), "wg_end_median_by_xcd(b%8)": by_xcd, "start_min_med_max": q(rel[:, 0]), "staged": q(rel[:, 1]),
               "wave_end": q(ends), "wave_end_spread_in_wg": q(spread),
               "kernel_span_us": round(float(ends.max()), 2)}
    print(wl, res[wl], flush=True)
    w.free()
print(json.dumps(res))
