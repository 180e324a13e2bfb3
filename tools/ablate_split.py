#!/usr/bin/env python3
"""Is a split GCM (CTR kernel + GHASH-only kernel) worth it?  Back-to-back medians of the
config-2 seal with ablations (no GHASH / no AES / neither / prologue only) next to the CTR
kernel over the same 64 MiB."""
import json, os, sys, ctypes
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from bench import Workload
from cryptmpi_2022_amd import _native as N, aead
w = Workload("gcm1k", 0, seed=3)
L = N.lib()
key = bytes(range(16))
res = {}
def timeit(fn, n=4, rounds=7):
    ts = []
    for _ in range(rounds):
        fn(); torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n): fn()
        e1.record(); torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / n)
    ts.sort(); return round(ts[len(ts)//2] * 1000, 1)
modes = [(0, "full"), (1, "noghash"), (2, "noaes"), (3, "neither"), (8, "prologue"), (4, "full_coal"), (7, "neither_coal")]
if os.environ.get("LANE") == "1":  # the round-2 lane kernel's ablations
    modes = [(0, "full"), (16, "nomem"), (32, "noaes"), (48, "nomem_noaes"), (64, "noghash"), (80, "aes_only"),
             (96, "mem_only")]
for m, name in modes:
    L.cmpi_debug_set_gcm_ablation(m)
    res[name] = timeit(w.seal)
L.cmpi_debug_set_gcm_ablation(0)
# CTR over the same 64 MiB
wc = Workload("ctr1g", 0, seed=3)
n64 = 64 << 20
cb = (ctypes.c_uint8 * 16)(*([0] * 16))
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
P = lambda t: ctypes.c_void_p(t.data_ptr())
res["ctr_64MiB"] = timeit(lambda: L.cmpi_ctr_xor(wc.ctx.handle, P(wc.ct), P(wc.pt), n64, cb, st))
print(json.dumps(res))
