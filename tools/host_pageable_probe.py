"""Pageable host-path seal rate against the CPU pack/unpack thread count (CMPI_HOST_THREADS is
read once per process, so run this once per setting):  CMPI_HOST_THREADS=16 python
tools/host_pageable_probe.py.  Prints bench.host_path_rate's JSON with the setting."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

if __name__ == "__main__":
    r = bench.host_path_rate(0)
    r["CMPI_HOST_THREADS"] = os.environ.get("CMPI_HOST_THREADS", "default")
    print(json.dumps(r), flush=True)
