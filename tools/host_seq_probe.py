#!/usr/bin/env python3
"""Host-path rate (bench.host_path_rate, pipelined pinned seal) in a fresh process, then again after
one bench.time_steps pass of config 2 — with the kernel-timing pass (hipExtLaunchKernel events) or
without it (CMPI_BENCH_NO_KPASS=1): does the timing pass leave the process's copies slower?"""
import json, os, sys, time
sys.path.insert(0, os.getcwd())
import torch, bench
r = {"kpass": os.environ.get("CMPI_BENCH_NO_KPASS") != "1"}
r["fresh"] = bench.host_path_rate(0)["host_api_pinned_pipelined_GiBps"]
w = bench.Workload("gcm1k", 0, seed=1)
w.seal(); w.open(); w.verify()
bench.time_steps(w, 100, 10, lambda: None, warmup_s=0.5)
w.free()
r["after_time_steps"] = bench.host_path_rate(0)["host_api_pinned_pipelined_GiBps"]
print(json.dumps(r))
