#!/usr/bin/env python3
"""Resident service, single host messages (page-locked): seal / open latency per message size for
each smallest chunk length (cmpi_debug_set_svc_ls_min: chunks of 64·2^ls blocks — fewer chunks
means fewer workgroups and cross-workgroup arrivals, more steps per wave), medians of 300."""
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
res = {}
for ls in (0, 1, 2, 3):
    L.cmpi_debug_set_svc_ls_min(ls)
    ctx = aead.AeadCtx(bytes(range(16)))
    ctx.service_start(20000)
    for n in (4096, 16384, 65536, 262144):
        pt = torch.randint(0, 256, (n,), dtype=torch.uint8).pin_memory()
        ct = torch.empty(n + 16, dtype=torch.uint8).pin_memory()
        back = torch.empty(n, dtype=torch.uint8).pin_memory()
        nn = torch.zeros(12, dtype=torch.uint8).pin_memory()
        st = ctypes.c_int32(0)
        P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        ts, to = [], []
        for _ in range(300):
            t0 = time.perf_counter()
            N.check(L.cmpi_gcm_seal_host(ctx.handle, P(ct), n + 16, P(pt), n, P(nn), 12, n, 1))
            t1 = time.perf_counter()
            N.check(L.cmpi_gcm_open_host(ctx.handle, P(back), n, P(ct), n + 16, P(nn), 12, n, 1, ctypes.byref(st)))
            t2 = time.perf_counter()
            ts.append(t1 - t0)
            to.append(t2 - t1)
        ok = bool(torch.equal(back, pt))
        res[f"ls{ls}_{n}"] = {"seal_us": round(float(np.median(ts)) * 1e6, 2), "open_us": round(float(np.median(to)) * 1e6, 2),
                              "ok": ok}
        print(ls, n, res[f"ls{ls}_{n}"], flush=True)
    ctx.service_stop()
    ctx.close()
print(json.dumps(res))
