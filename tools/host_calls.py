import sys, os, time, ctypes, json
sys.path.insert(0, os.getcwd())
import torch
import bench
from cryptmpi_2022_amd import _native as N, aead
n, nrec = 1024, 65536
pt = torch.randint(0, 256, (nrec * n,), dtype=torch.uint8).pin_memory()
nonces = torch.randint(0, 256, (nrec * 12,), dtype=torch.uint8).pin_memory()
out = torch.empty(nrec * (n + 16), dtype=torch.uint8).pin_memory()
ctx = aead.AeadCtx(bench.KEY, device=0)
L, h = N.lib(), ctx.handle
P = lambda t: ctypes.c_void_p(t.data_ptr())
d_pt = torch.empty(nrec * n, dtype=torch.uint8, device="cuda")
d_n = torch.empty(nrec * 12, dtype=torch.uint8, device="cuda")
d_ct = torch.empty(nrec * (n + 16), dtype=torch.uint8, device="cuda")
pre = os.environ.get("PRE", "")
if pre == "serial":  # what bench.host_path_rate runs first
    for _ in range(9):
        d_pt.copy_(pt, non_blocking=True)
        d_n.copy_(nonces, non_blocking=True)
        ctx.seal_batch(d_ct, d_pt, d_n, n, nrec)
        out.copy_(d_ct, non_blocking=True)
        torch.cuda.synchronize()
elif pre == "h2d":
    for _ in range(9):
        d_pt.copy_(pt, non_blocking=True)
        torch.cuda.synchronize()
elif pre == "d2h":
    for _ in range(9):
        out.copy_(d_ct, non_blocking=True)
        torch.cuda.synchronize()
ts = []
for i in range(12):
    t0 = time.perf_counter()
    N.check(L.cmpi_gcm_seal_host(h, P(out), n + 16, P(pt), n, P(nonces), 12, n, nrec))
    ts.append(round(nrec * n / (time.perf_counter() - t0) / 2**30, 1))
print(pre, json.dumps(ts))
