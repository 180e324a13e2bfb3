#!/usr/bin/env python3
"""In-process A/B of several builds of libcmpi_aead.so (tools/ab_build.sh): each library is
loaded with its own ctypes handle (RTLD_LOCAL), gets its own context on the same key, and the
variants are timed interleaved on identical device buffers (HIP events, median of rounds).
Outputs of every variant are compared byte for byte.
Usage: tools/ab_lib.py abtest/A/libcmpi_aead.so abtest/B/libcmpi_aead.so [--wl gcm1k,gcm4k,ctr1g,ocb1m]"""
import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from cryptmpi_2022_amd import _native  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("libs", nargs="+")
ap.add_argument("--wl", default="gcm1k,gcm4k,ctr1g,ocb1m")
ap.add_argument("--rounds", type=int, default=7)
args = ap.parse_args()

libs, names = [], []
for spec in args.libs:  # path[:sched] — the same .so may be loaded twice under different knobs
    p, _, sched = spec.partition(":")
    import shutil
    import tempfile

    path = os.path.abspath(p)
    if any(os.path.abspath(q.partition(":")[0]) == path for q in args.libs[: len(libs)]):
        tmp = os.path.join(tempfile.mkdtemp(), os.path.basename(path))  # distinct dlopen instance
        shutil.copy(path, tmp)
        path = tmp
    L = ctypes.CDLL(path)
    for name, (at, rt) in _native._SIGS.items():
        if hasattr(L, name):
            getattr(L, name).argtypes = at
            getattr(L, name).restype = rt
    if sched:
        L.cmpi_debug_set_sched(int(sched))
    libs.append(L)
    names.append(os.path.basename(os.path.dirname(os.path.abspath(p))) + (f"s{sched}" if sched else ""))

dev = torch.device("cuda:0")
key = bytes(range(16))
SHAPES = {"gcm1k": ("gcm", 65536, 1024), "gcm4k": ("gcm", 65536, 4096), "ocb1m": ("ocb", 4096, 1 << 20),
          "ctr1g": ("ctr", 1, 1 << 30), "a2a": ("gcm", 8, 1 << 20), "a2a64": ("gcm", 64, 1 << 20),
          "m4k": ("gcm", 1, 4096), "m64k": ("gcm", 1, 65536), "b8x4k": ("gcm", 8, 4096), "b256x4k": ("gcm", 256, 4096),
          "m1m": ("gcm", 1, 1 << 20), "b1024x16k": ("gcm", 1024, 16384)}


def ptr(t):
    return ctypes.c_void_p(t.data_ptr())


res = {}
for wl in args.wl.split(","):
    kind, nrec, n = SHAPES[wl]
    g = torch.Generator(device=dev).manual_seed(7)
    pt = torch.randint(0, 256, (nrec * n,), dtype=torch.uint8, device=dev, generator=g)
    nonces = torch.randint(0, 256, (nrec * 12,), dtype=torch.uint8, device=dev, generator=g)
    alg = {"gcm": 1, "ocb": 2, "ctr": 3}[kind]
    ctxs = [L.cmpi_ctx_new(alg, key, 16, 16, 0) for L in libs]
    outs = [torch.empty(nrec * (n + 16), dtype=torch.uint8, device=dev) for _ in libs]
    backs = [torch.empty(nrec * n, dtype=torch.uint8, device=dev) for _ in libs]
    status = torch.empty(nrec, dtype=torch.int32, device=dev)
    wss = []
    for L, c in zip(libs, ctxs):
        ws = 0
        if kind == "gcm":
            ws = L.cmpi_gcm_workspace_size(c, n, nrec)
        elif kind == "ocb":
            ws = L.cmpi_ocb_workspace_size(c, n, nrec)
        wss.append(torch.empty(max(ws, 16), dtype=torch.uint8, device=dev))
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    ctr_block = (ctypes.c_uint8 * 16)(*([0] * 12 + [0xff, 0xff, 0xff, 0x00]))

    def op(i, which):
        L, c = libs[i], ctxs[i]
        if kind == "ctr":
            src = pt if which == "seal" else outs[i]
            dst = outs[i] if which == "seal" else backs[i]
            return L.cmpi_ctr_xor(c, ptr(dst), ptr(src), n, ctr_block, stream)
        seal = L.cmpi_gcm_seal_batch if kind == "gcm" else L.cmpi_ocb_seal_batch
        opn = L.cmpi_gcm_open_batch if kind == "gcm" else L.cmpi_ocb_open_batch
        if which == "seal":
            return seal(c, ptr(outs[i]), n + 16, ptr(pt), n, ptr(nonces), 12, n, nrec, ptr(wss[i]), stream)
        return opn(c, ptr(backs[i]), n, ptr(outs[i]), n + 16, ptr(nonces), 12, n, nrec, ptr(status), ptr(wss[i]),
                   stream)

    times = {(i, w): [] for i in range(len(libs)) for w in ("seal", "open")}
    for rnd in range(args.rounds):
        for i in range(len(libs)):
            for w in ("seal", "open"):
                assert op(i, w) == 0
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(5):
                    op(i, w)
                e1.record()
                torch.cuda.synchronize()
                times[(i, w)].append(e0.elapsed_time(e1) / 5)
    same = all(torch.equal(outs[0][: nrec * (n + 16) if kind != "ctr" else n], o[: nrec * (n + 16) if kind != "ctr" else n])
               for o in outs[1:])
    rt = all(torch.equal(b, pt) for b in backs)
    row = {}
    for (i, w), t in times.items():
        t = sorted(t)
        med = t[len(t) // 2]
        row[f"{names[i]}_{w}"] = {
            "ms": round(med, 4), "GiBps": round(n * nrec / (med * 1e-3) / 2**30, 1)}
    row["outputs_identical"] = same
    row["round_trip"] = rt
    res[wl] = row
    print(json.dumps({wl: row}), flush=True)
    for L, c in zip(libs, ctxs):
        L.cmpi_ctx_free(c)
    del pt, outs, backs, wss
    torch.cuda.empty_cache()
