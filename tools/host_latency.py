#!/usr/bin/env python3
"""Single-message host-memory GCM seal+open latency through cmpi_gcm_seal_host /
cmpi_gcm_open_host (what the EVP drop-in and the 600 path call per MPI message): direct path
(kernel on page-locked host memory) vs the 3-stream DMA pipeline, pinned vs pageable buffers,
verified against each other and round-tripped."""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle  # noqa: E402
from cryptmpi_2022_amd import _native as N  # noqa: E402
from cryptmpi_2022_amd import aead  # noqa: E402

KEY = bytes(range(16))
L = N.lib()
ctx = aead.AeadCtx(KEY)
res = {}
for n in [int(x) for x in (sys.argv[1:] or ["1024", "4096", "65536", "262144", "1048576"])]:
    for mem in ("pinned", "pageable"):
        if mem == "pinned":
            pt, ct, bk = (torch.empty(m, dtype=torch.uint8).pin_memory() for m in (n, n + 16, n))
        else:
            pt, ct, bk = (torch.empty(m, dtype=torch.uint8) for m in (n, n + 16, n))
        pt.copy_(torch.randint(0, 256, (n,), dtype=torch.uint8))
        nonce = np.frombuffer(bytes(range(12)), np.uint8).copy()
        st = np.zeros(1, np.int32)
        P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        want = oracle.gcm_seal(KEY, bytes(nonce), pt.numpy().tobytes()) if n <= 65536 else None
        for direct, spin in ((1 << 30, 1), (1 << 30, 0), (0, 0)):
            L.cmpi_debug_set_host_direct(direct)
            L.cmpi_debug_set_host_spin(spin)

            def one():
                N.check(L.cmpi_gcm_seal_host(ctx.handle, P(ct), n + 16, P(pt), max(n, 1), nonce.ctypes.data, 12, n, 1))
                N.check(L.cmpi_gcm_open_host(ctx.handle, P(bk), max(n, 1), P(ct), n + 16, nonce.ctypes.data, 12, n, 1,
                                             st.ctypes.data))

            for _ in range(20):
                one()
            ok = bool(st[0] == 1 and torch.equal(bk, pt)) and (want is None or ct.numpy().tobytes() == want)
            ts = []
            for _ in range(5):
                t0 = time.perf_counter()
                for _ in range(50):
                    one()
                ts.append((time.perf_counter() - t0) / 50 * 1e6)
            key = f"{n}:{mem}:{('direct_spin' if spin else 'direct') if direct else 'pipeline'}"
            res[key] = {"seal_open_us": round(sorted(ts)[2], 2), "verified": ok}
            print(key, res[key], flush=True)
L.cmpi_debug_set_host_direct((2 << 20) + 64)
L.cmpi_debug_set_host_spin(1)
print(json.dumps(res))
