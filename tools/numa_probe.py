#!/usr/bin/env python3
"""Served-op and doorbell latencies per host NUMA node of the process (CPU affinity; page-locked
buffers are first-touched by the pinned threads, so they land on that node too).  The resident
service polls page-locked host memory and the host spins on words the GPU writes: a socket away
from the GPU's PCIe root adds its link to every round trip.  Runs tools/msg_latency per node."""
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
out = {}
try:
    import torch

    bus = torch.cuda.get_device_properties(0).pci_bus_id.lower() if hasattr(torch.cuda.get_device_properties(0), "pci_bus_id") else None
except Exception:
    bus = None
gpu_node = None
for path in glob.glob("/sys/bus/pci/devices/*/numa_node"):
    if bus and bus[-7:] in path:
        gpu_node = open(path).read().strip()
out["gpu_pci"] = bus
out["gpu_numa_node"] = gpu_node
nodes = sorted(int(p.rsplit("node", 1)[1]) for p in glob.glob("/sys/devices/system/node/node[0-9]*"))
for n in nodes:
    cpus = set()
    for part in open(f"/sys/devices/system/node/node{n}/cpulist").read().strip().split(","):
        a, _, b = part.partition("-")
        cpus.update(range(int(a), int(b or a) + 1))
    allowed = cpus & os.sched_getaffinity(0)
    if not allowed:
        out[f"node{n}"] = "no allowed cpus"
        continue
    p = subprocess.run([os.path.join(ROOT, "tools", "msg_latency"), "300"], capture_output=True, text=True, timeout=200,
                       preexec_fn=lambda c=sorted(allowed)[:16]: os.sched_setaffinity(0, c))
    if p.returncode:
        out[f"node{n}"] = p.stderr[-300:]
        continue
    d = json.loads(p.stdout.strip().splitlines()[-1])
    out[f"node{n}"] = {k: d.get(k) for k in ("flag_kernel_host_spin_us", "c702_4k_served_send_only_us", "c702_4k_served_recv_mask_us",
                                              "svc_pinned_seal_1k_us", "svc_pinned_seal_64k_us", "ctr_host_4k_served_us",
                                              "c702_4k_send_only_flag_us")}
    print(n, out[f"node{n}"], flush=True)
print(json.dumps(out))
