#!/bin/bash
# Round 4: the line-aligned lane stores at the bench's own clock — default bench headline (two
# overlapped streams) and --serial, hook off / on, interleaved, 3 rounds; no extras.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2 3; do
  for h in 0 1 2; do
    AB_HOOKS=lane_pair=$h timeout -k 10 120 python -u tools/bench_hooked.py --no-extras --no-cpu-baseline --steps 200 --warmup 50 >> gpurun_out/r04w_bench_pair$h.jsonl 2>> gpurun_out/r04w_bench.err
    AB_HOOKS=lane_pair=$h timeout -k 10 120 python -u tools/bench_hooked.py --no-extras --no-cpu-baseline --serial --steps 200 --warmup 50 >> gpurun_out/r04w_bench_serial_pair$h.jsonl 2>> gpurun_out/r04w_bench.err
    echo "round $r hook $h"
  done
done
