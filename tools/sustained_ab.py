#!/usr/bin/env python3
"""Interleaved A/B of two builds (or hook settings) of the engine at SUSTAINED clocks on a bench
workload: per (round, build) a fresh process runs 3 s of back-to-back seal + open steps (the
power-held regime of bench.py's timed region), then times 200 steps with fence-free HIP events
(seal and open kernel times separately) and checks the round trip.

    python tools/sustained_ab.py <libA.so[@hook=v,...]> <libB.so[@hook=v,...]> [more libs] [rounds] [workload]"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(workload: str) -> None:
    sys.path.insert(0, ROOT)
    import torch

    import bench
    from cryptmpi_2022_amd import _native as N

    for kv in filter(None, os.environ.get("AB_HOOKS", "").split(",")):
        k, v = kv.split("=")
        getattr(N.lib(), "cmpi_debug_set_" + k)(int(v))
    w = bench.Workload(workload, 0, seed=9)
    st = torch.cuda.current_stream().cuda_stream
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 3.0:
        for _ in range(16):
            w.seal()
            w.open()
        torch.cuda.synchronize()
    iters = 200
    ev = bench.KernelEvents(2 * iters + 1)
    ev.record(0, st)
    for i in range(iters):
        w.seal()
        ev.record(2 * i + 1, st)
        w.open()
        ev.record(2 * i + 2, st)
    torch.cuda.synchronize()
    seal = sum(ev.ms(2 * i, 2 * i + 1) for i in range(iters)) / iters * 1e3
    opn = sum(ev.ms(2 * i + 1, 2 * i + 2) for i in range(iters)) / iters * 1e3
    # the same steps with no event between the launches (two events around the whole run)
    ev.record(0, st)
    for i in range(iters):
        w.seal()
        w.open()
    ev.record(1, st)
    torch.cuda.synchronize()
    bare = ev.ms(0, 1) / iters * 1e3
    print(json.dumps({"seal_us": seal, "open_us": opn, "step_ms": (seal + opn) / 1e3, "step_us_no_events": bare,
                      "ok": bool(w.verify())}))


def main() -> None:
    if sys.argv[1] == "--child":
        child(sys.argv[2])
        return
    args = sys.argv[1:]
    libs = [x for x in args if ".so" in x]  # two or more builds
    rest = [x for x in args if ".so" not in x]
    rounds = int(rest[0]) if rest else 3
    workload = rest[1] if len(rest) > 1 else "gcm1k"
    runs = {lib: [] for lib in libs}
    for _ in range(rounds):
        for lib in libs:
            path, _, hooks = lib.partition("@")
            env = dict(os.environ, CMPI_LIB=os.path.abspath(path), CMPI_LIB_LENIENT="1", AB_HOOKS=hooks)
            p = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", workload], env=env,
                               capture_output=True, text=True, timeout=120)
            if p.returncode != 0:
                sys.stderr.write(p.stderr)
                sys.exit(p.returncode)
            r = json.loads(p.stdout.strip().splitlines()[-1])
            runs[lib].append(r)
            print(lib, r, flush=True)
    res = {}
    for lib in libs:
        s = sorted(r["seal_us"] for r in runs[lib])
        o = sorted(r["open_us"] for r in runs[lib])
        b = sorted(r["step_us_no_events"] for r in runs[lib])
        res[lib] = {"seal_us": round(s[len(s) // 2], 2), "open_us": round(o[len(o) // 2], 2),
                    "step_us_no_events": round(b[len(b) // 2], 2), "ok": all(r["ok"] for r in runs[lib])}
    print(json.dumps({"workload": workload, "rounds": rounds, "medians": res}))


if __name__ == "__main__":
    main()
