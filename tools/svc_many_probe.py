#!/usr/bin/env python3
"""Several contexts with resident message services in one process (the EVP shim with
CMPI_EVP_SERVICE_US: one service per key context): round-robin single 1 KiB host seals over K
contexts, per-call latency quantiles (a context whose service stream shares a hardware queue
with another resident service waits for that kernel to idle out)."""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from cryptmpi_2022_amd import _native as N  # noqa: E402
from cryptmpi_2022_amd import aead  # noqa: E402

L = N.lib()
n = 1024
res = {}
for K in (1, 3, 4, 5, 6, 8):
    ctxs = [aead.AeadCtx(bytes([k] * 16)) for k in range(K)]
    for c in ctxs:
        c.service_start(20000)
    pt = torch.randint(0, 256, (n,), dtype=torch.uint8).pin_memory()
    out = torch.empty(n + 16, dtype=torch.uint8).pin_memory()
    nn = torch.zeros(12, dtype=torch.uint8).pin_memory()
    lat = []
    t_all = time.perf_counter()
    for i in range(40 * K):
        c = ctxs[i % K]
        t0 = time.perf_counter()
        N.check(L.cmpi_gcm_seal_host(c.handle, ctypes.c_void_p(out.data_ptr()), n + 16, ctypes.c_void_p(pt.data_ptr()),
                                     n, ctypes.c_void_p(nn.data_ptr()), 12, n, 1))
        lat.append((time.perf_counter() - t0) * 1e6)
        if time.perf_counter() - t_all > 20:
            break
    lat = np.array(lat[K:])  # first call per context launches its kernel
    res[K] = {"calls": int(lat.size), "p50_us": round(float(np.median(lat)), 1), "p99_us": round(float(np.percentile(lat, 99)), 1),
              "max_us": round(float(lat.max()), 1)}
    print(K, res[K], flush=True)
    for c in ctxs:
        c.service_stop()
        c.close()
print(json.dumps(res))
