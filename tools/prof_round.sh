#!/bin/bash
# One round's profile set on a GPU box (run from the repo root through gpurun):
#  1. the default bench.py under rocprofv3 --kernel-trace --stats (every kernel of every workload)
#  2. PMC passes of the config-2 seal (tools/gpu_pmc.sh: one counter group per pass, --kernel-trace only)
#  3. the 602 8 MiB message rates under --kernel-trace --stats (re-key / seal / combine split)
# Outputs under gpurun_out/; summaries are copied into profiles/ by hand.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=${ROUND:-r04}
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${R}_bench -o run -- \
    python3 bench.py > gpurun_out/${R}_bench_under_rocprof.json 2> gpurun_out/${R}_bench_under_rocprof.err
echo BENCH_PROF_DONE
WL=gcm1k timeout -k 10 400 bash tools/gpu_pmc.sh
echo PMC_DONE
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${R}_602 -o run -- \
    python3 tools/framed_rates.py > gpurun_out/${R}_framed_rates_under_rocprof.json 2>&1
echo PROF_DONE
