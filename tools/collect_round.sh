#!/bin/bash
# Copy one validation pass's results (tools/val_round.sh, ROUND=<R>) from gpurun_out/ into
# profiles/ under the names DESIGN.md cites: tools/collect_round.sh <R> <name prefix, e.g. r06>
set -euo pipefail
R=$1; P=$2
cd "$(dirname "$0")/.."
o=gpurun_out
cp $o/${R}_bench.json profiles/${P}_bench.json
tail -3 $o/${R}_gpu_tests.log > profiles/${P}_gpu_tests_tail.txt
cp $o/${R}_smoke.log profiles/${P}_smoke.txt
cp $o/${R}_msg_latency.json profiles/${P}_msg_latency.json
if [ -d $o/prof_${R}_headline ]; then
  cp $o/prof_${R}_headline/run_kernel_stats.csv profiles/${P}_rocprof_headline_stats.csv
  python3 tools/rocprof_split.py $o/prof_${R}_headline/run_kernel_trace.csv \
    "${R}: bench.py --no-extras under rocprofv3 --kernel-trace --stats (line: profiles/${P}_headline_under_rocprof.json)" \
    > profiles/${P}_rocprof_headline_split.txt
  cp $o/${R}_headline_under_rocprof.json profiles/${P}_headline_under_rocprof.json
fi
if [ -d $o/prof_${R}_bench ]; then
  cp $o/prof_${R}_bench/run_kernel_stats.csv profiles/${P}_rocprof_bench_stats.csv
  python3 tools/rocprof_split.py $o/prof_${R}_bench/run_kernel_trace.csv \
    "${R}: default bench.py under rocprofv3 --kernel-trace --stats, split by schedule phase" \
    > profiles/${P}_rocprof_bench_split.txt
  cp $o/${R}_bench_under_rocprof.json profiles/${P}_bench_under_rocprof.json
fi
if [ -d $o/${R}_pmc_gcm1k ]; then
  ROUND="${R} (last 5 launches per pass after prof_driver's 0.5 s warm-up)" LAST=5 \
    python3 tools/pmc_summarize.py gcm1k $o/${R}_pmc_gcm1k "gcm_lane_kernel<4, false" > /dev/null
fi
echo collected $R as $P
