#!/usr/bin/env python3
"""Hardware-queue sharing probe: how the library's host
paths and its resident message service behave next to other streams of the same process.

HIP maps streams onto at most GPU_MAX_HW_QUEUES hardware queues (4 on the test box); two streams
on one queue run in submission order.  One process per (stream mode, scenario):
  mode      cmpi_debug_set_stream_mode: 0 non-blocking, 1 greatest priority, 2 CU-masked queue
  scenario  fresh        nothing else created
            torch1       one torch.cuda.Stream() created and used first (what bench.Pipeline does)
            hip32        32 extra hipStreams created first (an MPI process with other GPU users)
Measures: the pinned 65 536 x 1 KiB seal through cmpi_gcm_seal_host (the bench's
host_api_pinned_pipelined), an 8 MiB 602 message sealed from page-locked memory (one request per
outer message, all begun before the first wait), and — with the message service resident — the
completion latency of a tiny kernel on each of 8 other streams.
Usage: queue_probe.py --mode M --scenario S   (prints one JSON line);  queue_probe.py --all"""
import argparse
import ctypes
import json
import os
import subprocess
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

GIB = float(1 << 30)


def run(mode: int, scenario: str) -> dict:
    import numpy as np
    import torch

    from cryptmpi_2022_amd import _native as N
    from cryptmpi_2022_amd import aead, frame

    L = N.lib()
    L.cmpi_debug_set_stream_mode(mode)
    torch.cuda.init()
    keep = []
    if scenario == "torch1":
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            torch.ones(16, device="cuda").add_(1)
        keep.append(s)
    elif scenario == "hip32":
        hip = ctypes.CDLL("libamdhip64.so")
        for _ in range(32):
            st = ctypes.c_void_p()
            assert hip.hipStreamCreate(ctypes.byref(st)) == 0
            keep.append(st)
    torch.cuda.synchronize()
    res = {"mode": mode, "scenario": scenario}
    # (a) host_api pinned, 65 536 x 1 KiB seal
    n, nrec = 1024, 65536
    pt = torch.randint(0, 256, (nrec * n,), dtype=torch.uint8).pin_memory()
    nonces = torch.randint(0, 256, (nrec * 12,), dtype=torch.uint8).pin_memory()
    out = torch.empty(nrec * (n + 16), dtype=torch.uint8).pin_memory()
    ctx = aead.AeadCtx(bytes(range(16)))
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731

    def seal():
        N.check(L.cmpi_gcm_seal_host(ctx.handle, P(out), n + 16, P(pt), n, P(nonces), 12, n, nrec))

    for _ in range(3):
        seal()
    t0 = time.perf_counter()
    for _ in range(8):
        seal()
    res["host_api_pinned_GiBps"] = round(nrec * n * 8 / (time.perf_counter() - t0) / GIB, 2)
    # (b) 602 8 MiB message from page-locked memory, pipelined outer messages
    m = 8 << 20
    plan = frame.plan602(m, 8, 0)
    header = frame.header602(plan, bytes(range(16, 32)))
    seg = aead.AeadCtx(bytes(16))
    seg.rekey_subkey(ctx, header[4:20], stream=torch.cuda.current_stream())
    torch.cuda.synchronize()
    src = torch.randint(0, 256, (m,), dtype=torch.uint8).pin_memory().numpy()
    hw = torch.empty(plan.wire_bytes, dtype=torch.uint8).pin_memory().numpy()

    def s602():
        reqs = [frame.seal602_host_begin(seg, plan, header, hw, src, o) for o in range(plan.outer)]
        for q in reqs:
            q.wait()

    for _ in range(3):
        s602()
    best = float("inf")
    for _ in range(8):
        t0 = time.perf_counter()
        s602()
        best = min(best, time.perf_counter() - t0)
    res["seal602_pinned_pipelined_GiBps"] = round(m / best / GIB, 2)
    # (c) the resident service next to 8 other streams: completion latency of a tiny kernel each
    ctx.service_start(200000)  # 200 ms idle: resident through the measurement
    msg = np.zeros(4096, np.uint8)
    ctx.seal(bytes(12), msg.tobytes())
    assert ctx.service_running()
    streams = [torch.cuda.Stream() for _ in range(8)]
    x = torch.ones(16, device="cuda")
    lat = []
    for s in streams:
        t0 = time.perf_counter()
        with torch.cuda.stream(s):
            x.add_(1)
        s.synchronize()
        lat.append((time.perf_counter() - t0) * 1e6)
    t0 = time.perf_counter()
    torch.ones(16, device="cuda").add_(1)  # the legacy default stream
    torch.cuda.current_stream().synchronize()
    res["svc_default_stream_us"] = round((time.perf_counter() - t0) * 1e6, 1)
    res["svc_running_after"] = bool(ctx.service_running())
    ctx.service_stop()
    res["svc_other_stream_us"] = [round(v, 1) for v in lat]
    res["svc_other_stream_max_us"] = round(max(lat), 1)
    seg.close()
    ctx.close()
    return res


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", type=int, default=0)
    ap.add_argument("--scenario", default="fresh")
    ap.add_argument("--all", action="store_true")
    a = ap.parse_args()
    if not a.all:
        print(json.dumps(run(a.mode, a.scenario)), flush=True)
        return
    for mode in (0, 1, 2):
        for sc in ("fresh", "torch1", "hip32"):
            r = subprocess.run([sys.executable, os.path.abspath(__file__), "--mode", str(mode), "--scenario", sc],
                               capture_output=True, text=True, timeout=120)
            line = r.stdout.strip().splitlines()[-1] if r.stdout.strip() else json.dumps(
                {"mode": mode, "scenario": sc, "rc": r.returncode, "err": r.stderr[-800:]})
            print(line, flush=True)


if __name__ == "__main__":
    main()
