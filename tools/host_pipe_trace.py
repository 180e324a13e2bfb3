#!/usr/bin/env python3
"""The pipelined host path (cmpi_gcm_seal_host, 65 536 x 1 KiB from / to registered host buffers,
bench extras.host_path_pcie) for a rocprofv3 --kernel-trace --memory-copy-trace timeline, and the
timeline's summary: run it under rocprofv3, then `host_pipe_trace.py --summarize <trace dir>`.

    rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d D -o run -- python3 tools/host_pipe_trace.py
    python3 tools/host_pipe_trace.py --summarize D
    python3 tools/host_pipe_trace.py --detail D 40     (the last 40 events with queue / stream ids)

(CHUNK_MIB / OUT_DIRECT in the environment: the pipeline's chunk size and copy mode, default 5.)

The summary takes the last call: per chunk the H2D copy, kernel and D2H copy intervals (us from
the call's first copy), and the totals: the call's span, each engine's busy time, and the time
when both directions copied at once."""
import csv
import ctypes
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(calls: int = 6) -> None:
    sys.path.insert(0, ROOT)
    import torch

    import bench
    from cryptmpi_2022_amd import _native as N
    from cryptmpi_2022_amd import aead

    n, nrec = 1024, 65536
    pt = bench.registered_host_buffer(nrec * n)
    pt.copy_(torch.randint(0, 256, (nrec * n,), dtype=torch.uint8))
    nonces = bench.registered_host_buffer(nrec * 12)
    out = bench.registered_host_buffer(nrec * (n + 16))
    ctx = aead.AeadCtx(bench.KEY, device=0)
    L, h = N.lib(), ctx.handle
    if os.environ.get("CHUNK_MIB"):  # pipeline settings under test (cmpi_debug_set_host_chunk / _out_direct)
        L.cmpi_debug_set_host_chunk(int(os.environ["CHUNK_MIB"]) << 20)
    L.cmpi_debug_set_host_out_direct(int(os.environ.get("OUT_DIRECT", "5")))
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    rates = []
    for _ in range(calls):
        t0 = time.perf_counter()
        N.check(L.cmpi_gcm_seal_host(h, P(out), n + 16, P(pt), n, P(nonces), 12, n, nrec))
        rates.append(nrec * n / (time.perf_counter() - t0) / 2**30)
    print(json.dumps({"GiBps_per_call": [round(r, 2) for r in rates]}))


def summarize(d: str) -> None:
    def rows(pat):
        f = glob.glob(os.path.join(d, "**", pat), recursive=True)
        return list(csv.DictReader(open(f[0]))) if f else []

    cp = rows("*memory_copy_trace.csv")
    # the library's kernels, and HIP's blit kernels (a D2H copy into page-locked memory runs as
    # __amd_rocclr_copyBuffer, not on a copy engine)
    kt = [r for r in rows("*kernel_trace.csv") if "cmpi::dev" in r["Kernel_Name"] or "__amd_rocclr_copyBuffer" in r["Kernel_Name"]]
    ev = [("copy", r.get("Direction", r.get("Operation", "?")), int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
           int(r.get("Bytes", r.get("Size", 0)) or 0)) for r in cp]
    ev += [("kernel", r["Kernel_Name"].split("(")[0].replace("void cmpi::dev::", ""), int(r["Start_Timestamp"]),
            int(r["End_Timestamp"]), 0) for r in kt]
    ev.sort(key=lambda e: e[2])
    # the last call: the events after the last gap of > 2 ms
    start = 0
    for i in range(1, len(ev)):
        if ev[i][2] - max(e[3] for e in ev[:i]) > 2_000_000:
            start = i
    last = ev[start:]
    t0 = last[0][2]
    for kind, what, s, e, b in last:
        print(f"{kind:6s} {what[:40]:40s} {(s - t0) / 1e3:9.1f} .. {(e - t0) / 1e3:9.1f} us  {b / 2**20:7.2f} MiB")
    span = (max(e[3] for e in last) - t0) / 1e3

    def busy(sel):
        iv = sorted((s, e) for k, w, s, e, _ in last if sel(k, w))
        tot, cur = 0, None
        for s, e in iv:
            if cur is None or s > cur[1]:
                if cur:
                    tot += cur[1] - cur[0]
                cur = [s, e]
            else:
                cur[1] = max(cur[1], e)
        return (tot + (cur[1] - cur[0] if cur else 0)) / 1e3, iv

    h2d, iv_h = busy(lambda k, w: k == "copy" and "HOST_TO_DEVICE" in w.upper())
    d2h, iv_d = busy(lambda k, w: (k == "copy" and "DEVICE_TO_HOST" in w.upper()) or "__amd_rocclr" in w)
    kern, _ = busy(lambda k, w: k == "kernel" and "__amd_rocclr" not in w)
    both = 0
    for s1, e1 in iv_h:
        for s2, e2 in iv_d:
            both += max(0, min(e1, e2) - max(s1, s2))
    print(json.dumps({"span_us": round(span, 1), "h2d_busy_us": round(h2d, 1), "d2h_busy_us": round(d2h, 1),
                      "kernel_busy_us": round(kern, 1), "both_directions_us": round(both / 1e3, 1)}))


def detail(d: str, n: int) -> None:
    """The last n events of the trace (library kernels, HIP blit kernels, copies) with their queue
    and stream ids: start, end, duration in us from the first one shown."""
    def rows(pat):
        f = glob.glob(os.path.join(d, "**", pat), recursive=True)
        return list(csv.DictReader(open(f[0]))) if f else []

    ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:40], r.get("Queue_Id", ""),
           r.get("Stream_Id", "")) for r in rows("*kernel_trace.csv") if "fillBuffer" not in r["Kernel_Name"]]
    ev += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "COPY " + r.get("Direction", r.get("Operation", "")),
            r.get("Queue_Id", ""), r.get("Stream_Id", "")) for r in rows("*memory_copy_trace.csv")]
    ev.sort()
    t0 = ev[-n][0]
    for s, e, name, q, st in ev[-n:]:
        print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f} {name:40s} q={q} s={st}")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--summarize":
        summarize(sys.argv[2])
    elif len(sys.argv) > 3 and sys.argv[1] == "--detail":
        detail(sys.argv[2], int(sys.argv[3]))
    else:
        run()
