#!/bin/bash
# Round 4: the served-op and doorbell latencies per host NUMA placement (CPU + memory node of the
# process) — the resident service polls page-locked host memory and the host spins on a word the
# GPU writes, so both cross PCIe, and a remote socket adds its link to each round trip.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for f in /sys/class/drm/card*/device/numa_node; do echo "$f $(cat $f)"; done > gpurun_out/r04zu_numa_topo.txt 2>&1
(command -v numactl && numactl --hardware) >> gpurun_out/r04zu_numa_topo.txt 2>&1
nodes=$(ls -d /sys/devices/system/node/node* 2>/dev/null | sed 's/.*node//' | sort -n)
echo "nodes: $nodes" >> gpurun_out/r04zu_numa_topo.txt
for n in $nodes; do
  timeout -k 10 120 numactl --cpunodebind=$n --membind=$n tools/msg_latency 300 > gpurun_out/r04zu_numa_$n.json 2>/dev/null || echo "node $n failed" >> gpurun_out/r04zu_numa_topo.txt
done
echo done
