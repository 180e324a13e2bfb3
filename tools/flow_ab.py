#!/usr/bin/env python3
"""Interleaved A/B of two builds of the engine on the FLOW-kernel shapes (config 5's 8 x 1 MiB,
single 64 KiB messages, 3 x 100000 B, 1 x 8 MiB, 32 x 256 KiB) and two ragged ones (8 x (1 MiB - 5),
65536 x 1000 B on the lane kernel) and short records (1000 B, 100 B; few of them).

    [AB_SHAPES=65536x1024,65536x4096] python tools/flow_ab.py <libA.so> <libB.so> [rounds]
    (a build may carry test hooks: path/libcmpi_aead.so@lane_pair=0 calls
     cmpi_debug_set_lane_pair(0) in that build's processes; force_wide=1:8 calls
     cmpi_debug_force_wide(1, 8))

Each (round, build) runs in its own process (`--child <lib>`): per shape, 0.3 s of warm-up, then
seal and open kernel times from fence-free HIP events over 30 back-to-back calls; the parent prints
per-build medians and checks that both builds produced identical ciphertext."""
import hashlib
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHAPES = {"8x1MiB": (1 << 20, 8), "1x64KiB": (65536, 1), "3x100000": (100000, 3), "1x8MiB": (8 << 20, 1),
          "32x256KiB": (256 << 10, 32), "8x(1MiB-5)": ((1 << 20) - 5, 8), "65536x1000": (1000, 65536),
          "1x1000": (1000, 1), "64x1000": (1000, 64), "2048x1000": (1000, 2048), "16x100": (100, 16),
          "1x100": (100, 1), "2048x600": (600, 2048), "2048x300": (300, 2048), "2048x200": (200, 2048),
          "256x260": (260, 256), "16x300": (300, 16), "65536x1024": (1024, 65536), "65536x4096": (4096, 65536),
          "3000x1024": (1024, 3000), "4096x1024": (1024, 4096), "6000x1024": (1024, 6000), "2500x4000": (4000, 2500)}


def shapes() -> dict:
    """SHAPES, or the comma-separated subset named by AB_SHAPES."""
    sel = [x for x in os.environ.get("AB_SHAPES", "").split(",") if x]
    return {k: v for k, v in SHAPES.items() if not sel or k in sel}


def child() -> None:
    sys.path.insert(0, ROOT)
    import torch

    import bench
    from cryptmpi_2022_amd import _native as N

    for kv in filter(None, os.environ.get("AB_HOOKS", "").split(",")):
        k, v = kv.split("=")  # set_<k>(v), or force_<k>(a, b) for "force_wide=1:8"
        args = [int(x) for x in v.split(":")]
        getattr(N.lib(), "cmpi_debug_" + (k if k.startswith("force_") else "set_" + k))(*args)

    out = {}
    for name, (n, nrec) in shapes().items():
        bench.WORKLOADS["_ab"] = ("gcm", n, nrec, name)
        w = bench.Workload("_ab", 0, seed=5)
        st = torch.cuda.current_stream().cuda_stream
        iters = 30
        ev = bench.KernelEvents(2 * iters + 1)
        t_w = time.perf_counter()
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
        seal = sum(ev.ms(2 * i, 2 * i + 1) for i in range(iters)) / iters * 1e3
        opn = sum(ev.ms(2 * i + 1, 2 * i + 2) for i in range(iters)) / iters * 1e3
        ok = w.verify()
        out[name] = {"seal_us": seal, "open_us": opn, "ok": ok,
                     "ct_sha": hashlib.sha256(w.ct.cpu().numpy().tobytes()).hexdigest()[:16]}
        ev.free()
        w.free()
    print(json.dumps(out))


def main() -> None:
    if sys.argv[1] == "--child":
        child()
        return
    libs = sys.argv[1:3]
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    runs = {lib: [] for lib in libs}
    for _ in range(rounds):
        for lib in libs:
            path, _, hooks = lib.partition("@")
            env = dict(os.environ, CMPI_LIB=os.path.abspath(path), CMPI_LIB_LENIENT="1", AB_HOOKS=hooks)
            p = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", lib], env=env,
                               capture_output=True, text=True, timeout=120)
            if p.returncode != 0:
                sys.stderr.write(p.stderr)
                sys.exit(p.returncode)
            runs[lib].append(json.loads(p.stdout.strip().splitlines()[-1]))
    res = {}
    for name in shapes():
        row = {}
        for lib in libs:
            s = sorted(r[name]["seal_us"] for r in runs[lib])
            o = sorted(r[name]["open_us"] for r in runs[lib])
            n, nrec = SHAPES[name]
            path, _, hooks = lib.partition("@")
            key = os.path.basename(os.path.dirname(os.path.abspath(path))) + "/" + os.path.basename(path)
            row[key + ("@" + hooks if hooks else "")] = {"seal_us": round(s[len(s) // 2], 2), "open_us": round(o[len(o) // 2], 2),
                                          "seal_GiBps": round(n * nrec / (s[len(s) // 2] * 1e-6) / (1 << 30), 1),
                                          "ok": all(r[name]["ok"] for r in runs[lib])}
        row["same_ct"] = len({r[name]["ct_sha"] for lib in libs for r in runs[lib]}) == 1
        res[name] = row
        print(name, row, flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
