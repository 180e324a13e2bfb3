#!/usr/bin/env python3
"""Where a small message's time goes: per-call wall time (host clock, synchronised every call) of
a device-resident GCM seal of one record, wide (FLOW + combine: two launches) vs lane-group plan
(one launch), next to an empty torch kernel launch + sync and the host-memory call."""
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
ctx = aead.AeadCtx(bytes(range(16)))
dev = torch.device("cuda", 0)
st = torch.cuda.current_stream(dev)
res = {}


def timeit(fn, reps=300):
    for _ in range(30):
        fn()
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        for _ in range(reps // 5):
            fn()
        ts.append((time.perf_counter() - t0) / (reps // 5) * 1e6)
    return round(sorted(ts)[2], 2)


x = torch.zeros(16, device=dev)
res["torch_add_sync_us"] = timeit(lambda: (x.add_(1), torch.cuda.synchronize()))
for n in (1024, 65536):
    pt = torch.randint(0, 256, (n,), dtype=torch.uint8, device=dev)
    ct = torch.empty(n + 16, dtype=torch.uint8, device=dev)
    nn = torch.arange(12, dtype=torch.uint8, device=dev)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731

    def seal():
        N.check(L.cmpi_gcm_seal_batch(ctx.handle, P(ct), n + 16, P(pt), n, P(nn), 12, n, 1, None, ctypes.c_void_p(st.cuda_stream)))
        torch.cuda.synchronize()

    def seal_nosync():
        N.check(L.cmpi_gcm_seal_batch(ctx.handle, P(ct), n + 16, P(pt), n, P(nn), 12, n, 1, None, ctypes.c_void_p(st.cuda_stream)))

    for mode in (0, -1):
        aead.force_wide(mode, 0)
        res[f"{n}:{'auto' if mode == 0 else 'lane'}"] = {"plan": aead.gcm_plan(ctx, n, 1), "seal_sync_us": timeit(seal),
                                                         "enqueue_only_us": timeit(seal_nosync)}
        torch.cuda.synchronize()
    aead.force_wide(0, 0)
print(json.dumps(res, indent=1))
