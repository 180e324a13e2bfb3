#!/usr/bin/env python3
"""bench.py with engine test hooks applied first (A/B of a hook at the bench's own clock):

    AB_HOOKS=lane_pair=1 python tools/bench_hooked.py --no-extras --no-cpu-baseline

Sets every cmpi_debug_set_<name>(value) of AB_HOOKS, then runs bench.py as __main__ in this
process with the remaining arguments (single rank only)."""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from cryptmpi_2022_amd import _native as N  # noqa: E402

for kv in filter(None, os.environ.get("AB_HOOKS", "").split(",")):
    k, v = kv.split("=")
    getattr(N.lib(), "cmpi_debug_set_" + k)(int(v))
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[1:]
runpy.run_path(sys.argv[0], run_name="__main__")
