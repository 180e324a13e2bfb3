"""Why bench.py's first serial pass timed config-2 seals at ~71 us while later passes (and
tools/sustained_ab.py) time ~60 us on the same box (round 5 diagnostic).  argv[1] selects what
runs before bench.time_steps in a fresh process:
  none     nothing (bench.py's order)
  verify   a Workload.verify() (torch ops) first
  deep     a 0.5 s warm-up enqueued without synchronising (deep queue)
  pass     one bench.time_steps pass first, report the second"""
import sys, time
sys.path.insert(0, '.')
import torch, bench

mode = sys.argv[1]
w = bench.Workload("gcm1k", 0, seed=1000)
if mode == "verify":
    w.seal(); w.open(); w.verify()
elif mode == "deep":
    t = time.perf_counter()
    while time.perf_counter() - t < 0.5:
        w.seal(); w.open()
    torch.cuda.synchronize()
elif mode == "pass":
    bench.time_steps(w, 100, 10, lambda: None, warmup_s=0.5)
wall, seal_ms, open_ms = bench.time_steps(w, 100, 10, lambda: None, warmup_s=0.5)
print(mode, "seal_us", round(seal_ms * 1e3, 2), "open_us", round(open_ms * 1e3, 2), "wall_us_per_step", round(wall / 100 * 1e6, 1), flush=True)
