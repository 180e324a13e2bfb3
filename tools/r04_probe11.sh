#!/bin/bash
# Round 4: PMC passes of the default build (line-aligned lane stores) on configs 2 and the 4 KiB
# workload, summarised like round 3's profiles/pmc_<wl>.json.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PMC_OUT=gpurun_out/r04x_pmc_gcm1k WL=gcm1k timeout -k 10 400 bash tools/gpu_pmc.sh
echo PMC1
PMC_OUT=gpurun_out/r04x_pmc_gcm4k WL=gcm4k timeout -k 10 400 bash tools/gpu_pmc.sh
echo PMC2
