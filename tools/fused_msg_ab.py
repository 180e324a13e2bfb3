#!/usr/bin/env python3
"""Single messages (the per-message EVP / 600 regime), alternating variants of the flow kernel's
tag finish: "combine" (XOR-combine launch), "fused" (last-arriver atomics, cmpi_debug_set_flow
flags bit 0), "one_wg" (a batch in one workgroup finishes its tags from LDS, in-kernel zero-fill;
cmpi_debug_set_flow_one_wg), "one_wg1024" (the same with 1024-thread workgroups kept, so up to
16 chunks fit one workgroup).  Device-resident seal / open (HIP events over 50 calls) and pinned
host seal+open (wall clock), every output checked against the oracle, plus a forged tag.
FMA_SIZES / FMA_VARIANTS (comma lists) select the cases."""
import ctypes
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle  # noqa: E402
from cryptmpi_2022_amd import _native as N, aead  # noqa: E402

KEY = bytes(range(16))
L = N.lib()
ctx = aead.AeadCtx(KEY)
P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
res = {}
VARIANTS = {"combine": (0, 0), "fused": (1, 0), "one_wg": (0, 1), "one_wg1024": (32, 1)}  # 32: keep 1024 threads
names = os.environ.get("FMA_VARIANTS", "combine,one_wg").split(",")
for n in [int(x) for x in os.environ.get("FMA_SIZES", "1024,4096,16384,65536").split(",")]:
    pt = torch.randint(0, 256, (n,), dtype=torch.uint8)
    nonce = torch.randint(0, 256, (12,), dtype=torch.uint8)
    want = oracle.gcm_seal(KEY, bytes(nonce.numpy()), pt.numpy().tobytes())
    d_pt, d_n = pt.cuda(), nonce.cuda()
    d_ct, d_bk = torch.empty(n + 16, dtype=torch.uint8, device="cuda"), torch.empty(n, dtype=torch.uint8, device="cuda")
    d_st = torch.zeros(1, dtype=torch.int32, device="cuda")
    h_pt, h_ct, h_bk = pt.pin_memory(), torch.empty(n + 16, dtype=torch.uint8).pin_memory(), torch.empty(n, dtype=torch.uint8).pin_memory()
    h_n = nonce.pin_memory()
    st = np.zeros(1, np.int32)
    t = {}
    for rep in range(7):
        for name in names:
            flags, one = VARIANTS[name]
            L.cmpi_debug_set_flow(1024, flags)
            L.cmpi_debug_set_flow_one_wg(one)
            e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
            ctx.seal_batch(d_ct, d_pt, d_n, n, 1)
            ctx.open_batch(d_bk, d_ct, d_n, n, 1, status=d_st)
            torch.cuda.synchronize()
            e0.record()
            ti = time.perf_counter()
            for _ in range(50):
                ctx.seal_batch(d_ct, d_pt, d_n, n, 1)
            issue_us = (time.perf_counter() - ti) / 50 * 1e6  # host time to submit, before any sync
            e1.record()
            for _ in range(50):
                ctx.open_batch(d_bk, d_ct, d_n, n, 1, status=d_st)
            e2.record()
            torch.cuda.synchronize()
            assert d_ct.cpu().numpy().tobytes() == want and int(d_st.item()) == 1
            t0 = time.perf_counter()
            for _ in range(50):
                N.check(L.cmpi_gcm_seal_host(ctx.handle, P(h_ct), n + 16, P(h_pt), n, P(h_n), 12, n, 1))
                N.check(L.cmpi_gcm_open_host(ctx.handle, P(h_bk), n, P(h_ct), n + 16, P(h_n), 12, n, 1, st.ctypes.data))
            host_us = (time.perf_counter() - t0) / 50 * 1e6
            assert h_ct.numpy().tobytes() == want and torch.equal(h_bk, pt)
            bad = d_ct.clone()
            bad[n] ^= 1
            d_bk.fill_(0x5A)
            ctx.open_batch(d_bk, bad, d_n, n, 1, status=d_st)
            torch.cuda.synchronize()
            assert int(d_st.item()) == 0 and not bool(d_bk.any()), "forged tag: status 0, zeroed output"
            if rep:
                for k, v in (("dev_seal_us", e0.elapsed_time(e1) / 50 * 1e3), ("dev_open_us", e1.elapsed_time(e2) / 50 * 1e3),
                             ("host_seal_open_us", host_us), ("seal_issue_us", issue_us)):
                    t.setdefault(f"{name}_{k}", []).append(v)
    L.cmpi_debug_set_flow(1024, 0)
    L.cmpi_debug_set_flow_one_wg(1)
    res[n] = {k: round(statistics.median(v), 2) for k, v in t.items()}
    print(n, res[n], flush=True)
print(json.dumps(res))
