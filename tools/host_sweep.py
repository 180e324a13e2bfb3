#!/usr/bin/env python3
"""Host-path sweep (diagnostics): PCIe-inclusive 65 536 x 1 KiB GCM seal on pinned host buffers —
the serial one-stream reference and cmpi_gcm_seal_host at several pipeline chunk sizes."""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from cryptmpi_2022_amd import _native as N, aead  # noqa: E402

GIB = 1 << 30
n, nrec = 1024, 65536
key = bytes(range(16))
ctx = aead.AeadCtx(key, device=0)
pt = torch.randint(0, 256, (nrec * n,), dtype=torch.uint8).pin_memory()
nonces = torch.randint(0, 256, (nrec * 12,), dtype=torch.uint8).pin_memory()
out = torch.empty(nrec * (n + 16), dtype=torch.uint8).pin_memory()
d_pt = torch.empty(nrec * n, dtype=torch.uint8, device="cuda")
d_n = torch.empty(nrec * 12, dtype=torch.uint8, device="cuda")
d_ct = torch.empty(nrec * (n + 16), dtype=torch.uint8, device="cuda")
L, h = N.lib(), ctx.handle
P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731


def serial():
    d_pt.copy_(pt, non_blocking=True)
    d_n.copy_(nonces, non_blocking=True)
    ctx.seal_batch(d_ct, d_pt, d_n, n, nrec)
    out.copy_(d_ct, non_blocking=True)
    torch.cuda.synchronize()


def host_api():
    N.check(L.cmpi_gcm_seal_host(h, P(out), n + 16, P(pt), n, P(nonces), 12, n, nrec))


def rate(fn, reps=8):
    fn()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    return round(nrec * n / ((time.perf_counter() - t0) / reps) / GIB, 2)


res = {"env_sdma": os.environ.get("HSA_ENABLE_SDMA", "default"), "serial": rate(serial)}
sizes = [int(x) for x in os.environ.get("SWEEP_MIB", "2,4,8,16,32").split(",")]
for mib in sizes:
    L.cmpi_debug_set_host_chunk(mib << 20)
    res[f"pipelined_{mib}MiB"] = rate(host_api)
L.cmpi_debug_set_host_chunk(0)
print(json.dumps(res), flush=True)
