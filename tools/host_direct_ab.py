#!/usr/bin/env python3
"""Host-memory GCM calls on page-locked buffers: the direct path (the kernel reads and writes the
host records itself over PCIe) against the chunked DMA pipeline (H2D | kernel | D2H), per batch
shape, alternating the two forms call by call.  Rates are plaintext GiB/s of one synchronous
cmpi_gcm_seal_host / cmpi_gcm_open_host call, median of the repetitions.

    python tools/host_direct_ab.py [shape ...]     shapes like 1024x65536 (bytes x records)
"""
import ctypes
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from cryptmpi_2022_amd import _native as N, aead  # noqa: E402

DEFAULT_DIRECT = (2 << 20) + 64
shapes = [tuple(int(v) for v in s.split("x")) for s in (sys.argv[1:] or ["1024x65536", "4096x16384", "1048576x64"])]
L = N.lib()
ctx = aead.AeadCtx(bench.KEY, device=0)
P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
res = {}
for n, nrec in shapes:
    pt = torch.randint(0, 256, (nrec * n,), dtype=torch.uint8).pin_memory()
    nonces = torch.randint(0, 256, (nrec * 12,), dtype=torch.uint8).pin_memory()
    ct = torch.empty(nrec * (n + 16), dtype=torch.uint8).pin_memory()
    back = torch.empty(nrec * n, dtype=torch.uint8).pin_memory()
    st = torch.zeros(nrec, dtype=torch.int32).pin_memory()
    t = {(f, op): [] for f in ("direct", "pipe") for op in ("seal", "open")}
    for rep in range(9):
        for form in ("direct", "pipe"):
            L.cmpi_debug_set_host_direct(ctypes.c_size_t(1 << 40) if form == "direct" else ctypes.c_size_t(DEFAULT_DIRECT))
            t0 = time.perf_counter()
            N.check(L.cmpi_gcm_seal_host(ctx.handle, P(ct), n + 16, P(pt), n, P(nonces), 12, n, nrec))
            t1 = time.perf_counter()
            N.check(L.cmpi_gcm_open_host(ctx.handle, P(back), n, P(ct), n + 16, P(nonces), 12, n, nrec, P(st)))
            t2 = time.perf_counter()
            if rep:  # the first repetition warms both forms (bounce buffers, staging slots)
                t[(form, "seal")].append(nrec * n / (t1 - t0) / 2**30)
                t[(form, "open")].append(nrec * n / (t2 - t1) / 2**30)
            assert torch.equal(back, pt) and bool((st == 1).all()), (form, n, nrec)
    L.cmpi_debug_set_host_direct(ctypes.c_size_t(DEFAULT_DIRECT))
    key = f"{nrec}x{n}"
    res[key] = {f"{f}_{op}_GiBps": round(statistics.median(v), 2) for (f, op), v in t.items()}
    print(key, res[key], flush=True)
    del pt, nonces, ct, back, st
print(json.dumps(res))
