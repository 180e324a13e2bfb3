#!/bin/bash
# Round-4 GPU pass 2: host-path regression probe, 602 host rates, C-timed message latencies (incl. 702)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u tools/host_regress_probe.py --all > gpurun_out/r04b_host_regress.jsonl 2> gpurun_out/r04b_host_regress.err || exit $?
timeout -k 10 200 tools/msg_latency 2000 > gpurun_out/r04b_msg_latency.json 2> gpurun_out/r04b_msg_latency.err || exit $?
echo ALL_DONE
