#!/usr/bin/env python3
"""Host-path regression probe: bench.host_path_rate (65 536 x 1 KiB seal from
page-locked / pageable memory through cmpi_gcm_seal_host) measured in a process that first ran
what the default bench runs before it, one scenario per process:
  fresh        nothing before
  serial       the headline workload's serial timed steps (time_steps)
  pipelined    + the two-stream pipelined steps (time_steps_pipelined: a second torch stream)
  extras       the bench's extra workloads alone (gcm4k, ocb1m, ctr1g, alltoall)
  config1      bench.config1_message alone (64 KiB messages, the resident service started / stopped)
  bench        pipelined + extras + config1: what the default bench runs before host_path_rate
and the 8 MiB 602 message from page-locked memory: one request per outer message (the pipelined
sender) with the CPU time of the 16 *_begin calls alone, and whole-message calls.
Usage: host_regress_probe.py --all   (one JSON line per scenario)"""
import argparse
import json
import os
import subprocess
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
GIB = float(1 << 30)


def f602(res: dict) -> None:
    import torch

    from cryptmpi_2022_amd import _native as N
    from cryptmpi_2022_amd import aead, frame

    m = 8 << 20
    plan = frame.plan602(m, 8, 0)
    header = frame.header602(plan, bytes(range(16, 32)))
    master = aead.AeadCtx(bytes(range(16)))
    seg = aead.AeadCtx(bytes(16))
    seg.rekey_subkey(master, header[4:20], stream=torch.cuda.current_stream())
    torch.cuda.synchronize()
    src = torch.randint(0, 256, (m,), dtype=torch.uint8).pin_memory().numpy()
    hw = torch.empty(plan.wire_bytes, dtype=torch.uint8).pin_memory().numpy()
    L = N.lib()
    back = torch.empty(m, dtype=torch.uint8).pin_memory().numpy()
    out = {}
    for form, span in (("direct", 16 << 20), ("dma", 0)):
        L.cmpi_debug_set_span_direct(span)
        o_form = {}
        for per in (1, 4, 16):
            begin_s = []

            def once():
                t0 = time.perf_counter()
                reqs = [frame.seal602_host_begin(seg, plan, header, hw, src, o, per) for o in range(0, plan.outer, per)]
                begin_s.append(time.perf_counter() - t0)
                for q in reqs:
                    q.wait()

            for _ in range(3):
                once()
            begin_s.clear()
            best = float("inf")
            for _ in range(8):
                t0 = time.perf_counter()
                once()
                best = min(best, time.perf_counter() - t0)
            o_form[f"seal_outer_per_request_{per}"] = {"GiBps": round(m / best / GIB, 2), "best_us": round(best * 1e6, 1),
                                                        "begin_calls_us_median": round(sorted(begin_s)[len(begin_s) // 2] * 1e6, 1)}

        def opn():
            reqs = [frame.open602_host_begin(seg, header, back, hw, o) for o in range(plan.outer)]
            for q in reqs:
                q.wait()

        def whole():
            frame.seal602_host(seg, plan, header, hw, src)

        for name, fn in (("open_outer_per_request_1", opn), ("seal_host_whole", whole)):
            for _ in range(3):
                fn()
            best = float("inf")
            for _ in range(8):
                t0 = time.perf_counter()
                fn()
                best = min(best, time.perf_counter() - t0)
            o_form[name + "_GiBps"] = round(m / best / GIB, 2)
        o_form["round_trip_ok"] = back.tobytes() == src.tobytes()
        out[form] = o_form
    L.cmpi_debug_set_span_direct(16 << 20)
    res["seal602_pinned"] = out
    del L
    seg.close()
    master.close()


def thp_buffer(nbytes: int):
    """nbytes of anonymous memory, 2 MiB aligned, madvise(MADV_HUGEPAGE), page-locked with
    hipHostRegister: a numpy view and the keep-alive (address)."""
    import ctypes

    import numpy as np

    libc = ctypes.CDLL(None)
    libc.mmap.restype = ctypes.c_void_p
    libc.mmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_long]
    libc.madvise.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    span = nbytes + (2 << 20)
    raw = libc.mmap(None, span, 3, 0x22, -1, 0)
    base = (raw + (2 << 20) - 1) & ~((2 << 20) - 1)
    libc.madvise(ctypes.c_void_p(base), nbytes, 14)  # MADV_HUGEPAGE
    a = np.frombuffer((ctypes.c_uint8 * nbytes).from_address(base), dtype=np.uint8)
    a[:] = 1  # fault the pages in (huge pages where the kernel has them)
    hip = ctypes.CDLL("libamdhip64.so")
    assert hip.hipHostRegister(ctypes.c_void_p(base), ctypes.c_size_t(nbytes), 0) == 0
    return a


def raw_dma(res: dict) -> None:
    """Raw pinned DMA bandwidth in this process state: 64 MiB H2D, D2H, and both at once on two
    streams (torch pin_memory buffers, then THP-backed registered buffers)."""
    import torch

    nb = 64 << 20
    d1 = torch.empty(nb, dtype=torch.uint8, device="cuda")
    d2 = torch.empty(nb, dtype=torch.uint8, device="cuda")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    out = {}
    for kind in ("torch_pin", "thp_registered"):
        if kind == "torch_pin":
            h1 = torch.empty(nb, dtype=torch.uint8).pin_memory()
            h2 = torch.empty(nb, dtype=torch.uint8).pin_memory()
        else:
            h1 = torch.from_numpy(thp_buffer(nb))
            h2 = torch.from_numpy(thp_buffer(nb))

        def t(fn, reps=5):
            fn()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                fn()
            torch.cuda.synchronize()
            return nb * reps / (time.perf_counter() - t0) / 1e9

        def both():
            with torch.cuda.stream(s1):
                d1.copy_(h1, non_blocking=True)
            with torch.cuda.stream(s2):
                h2.copy_(d2, non_blocking=True)

        out[kind] = {"h2d_GBps": round(t(lambda: d1.copy_(h1, non_blocking=True)), 2),
                     "d2h_GBps": round(t(lambda: h2.copy_(d2, non_blocking=True)), 2),
                     "duplex_each_GBps": round(t(both), 2)}
    res["raw_dma"] = out


def host_rate_thp(res: dict) -> None:
    """bench.host_path_rate's pinned leg on THP-backed registered buffers."""
    import ctypes

    import torch

    from cryptmpi_2022_amd import _native as N
    from cryptmpi_2022_amd import aead

    n, nrec = 1024, 65536
    pt, out, nn = thp_buffer(nrec * n), thp_buffer(nrec * (n + 16)), thp_buffer(nrec * 12)
    ctx = aead.AeadCtx(bytes(range(16)))
    L = N.lib()

    def f():
        N.check(L.cmpi_gcm_seal_host(ctx.handle, ctypes.c_void_p(out.ctypes.data), n + 16,
                                     ctypes.c_void_p(pt.ctypes.data), n, ctypes.c_void_p(nn.ctypes.data), 12, n, nrec))

    for _ in range(3):
        f()
    t0 = time.perf_counter()
    for _ in range(8):
        f()
    res["host_api_pinned_thp_GiBps"] = round(nrec * n * 8 / (time.perf_counter() - t0) / GIB, 2)
    ctx.close()
    del torch


def run(scenario: str) -> dict:
    import torch

    import bench

    res = {"scenario": scenario}
    torch.cuda.set_device(0)
    if scenario in ("serial", "pipelined", "bench"):
        w = bench.Workload("gcm1k", 0, seed=1000)
        bench.time_steps(w, 100, 10, lambda: None, warmup_s=0.5)
        if scenario in ("pipelined", "bench"):
            bench.time_steps_pipelined(w, 100, 10, lambda: None, warmup_s=0.2)
        w.free()
    if scenario in ("bench", "extras"):
        for name in ("gcm4k", "ocb1m", "ctr1g", "alltoall"):
            we = bench.Workload(name, 0, seed=77)
            bench.time_steps(we, 30, 10, lambda: None, warmup_s=0.3)
            we.free()
    if scenario in ("bench", "config1"):
        bench.config1_message(0)
    res["host_path_pcie"] = bench.host_path_rate(0)
    raw_dma(res)
    host_rate_thp(res)
    f602(res)
    return res


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--scenario", default="fresh")
    ap.add_argument("--all", action="store_true")
    a = ap.parse_args()
    if not a.all:
        print(json.dumps(run(a.scenario)), flush=True)
        return
    scen = os.environ.get("SCENARIOS", "fresh,pipelined,extras,config1,bench").split(",")
    for sc in scen:
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--scenario", sc], capture_output=True, text=True,
                           timeout=240)
        line = r.stdout.strip().splitlines()[-1] if r.stdout.strip() else json.dumps(
            {"scenario": sc, "rc": r.returncode, "err": r.stderr[-800:]})
        print(line, flush=True)


if __name__ == "__main__":
    main()
