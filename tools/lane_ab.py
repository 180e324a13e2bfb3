#!/usr/bin/env python3
"""Interleaved A/B of a lane-kernel test hook on the bench workloads (config 2 and the 4 KiB
target): per arm, seal and open kernel times from fence-free HIP events over `iters` back-to-back
steps, arms interleaved over `rounds` (medians); outputs must be identical across arms.
usage: tools/lane_ab.py <hook> <value,value,...> [workloads]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from cryptmpi_2022_amd import _native as N  # noqa: E402


def main():
    hook = sys.argv[1]
    vals = [int(v) for v in sys.argv[2].split(",")]
    wls = sys.argv[3].split(",") if len(sys.argv) > 3 else ["gcm1k", "gcm4k"]
    L = N.lib()
    set_ = getattr(L, hook)
    iters, rounds = 30, 7
    res = {}
    for wl in wls:
        w = bench.Workload(wl, 0, seed=11)
        st = torch.cuda.current_stream().cuda_stream
        ev = bench.KernelEvents(2 * iters + 1)
        arms = {v: {"seal_us": [], "open_us": []} for v in vals}
        ref = None
        for r in range(rounds):
            for v in vals:
                set_(v)
                t_w = time.perf_counter()  # >= 0.3 s of warm-up per arm: clocks at steady state
                while time.perf_counter() - t_w < 0.3:
                    for _ in range(8):
                        w.seal()
                        w.open()
                    torch.cuda.synchronize()
                ev.record(0, st)
                for i in range(iters):
                    w.seal()
                    ev.record(2 * i + 1, st)
                    w.open()
                    ev.record(2 * i + 2, st)
                torch.cuda.synchronize()
                arms[v]["seal_us"].append(sum(ev.ms(2 * i, 2 * i + 1) for i in range(iters)) / iters * 1e3)
                arms[v]["open_us"].append(sum(ev.ms(2 * i + 1, 2 * i + 2) for i in range(iters)) / iters * 1e3)
                h = hash(w.ct.cpu().numpy().tobytes())
                assert w.verify(), (wl, v)
                ref = h if ref is None else ref
                assert h == ref, ("output differs", wl, v)
        set_(vals[0])
        out = {}
        for v, a in arms.items():
            s, o = sorted(a["seal_us"]), sorted(a["open_us"])
            out[str(v)] = {"seal_us": round(s[len(s) // 2], 2), "open_us": round(o[len(o) // 2], 2),
                           "seal_GiBps": round(w.n * w.nrec / (s[len(s) // 2] * 1e-6) / (1 << 30), 1),
                           "open_GiBps": round(w.n * w.nrec / (o[len(o) // 2] * 1e-6) / (1 << 30), 1)}
        res[wl] = out
        print(wl, out, flush=True)
        ev.free()
        w.free()
    print(json.dumps({"hook": hook, "results": res}))


if __name__ == "__main__":
    main()
