#!/bin/bash
# Round 4: the lane kernel's paired main loop (cmpi_debug_set_lane_pair) — parity, A/B timing on
# the lane shapes, and the HBM write counters of both forms on config 2 (65 536 x 1 KiB seal).
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_gcm.py > gpurun_out/r04u_gcm_tests.log 2>&1
echo TESTS_DONE
timeout -k 10 500 python -u tools/flow_ab.py ab/pair/libcmpi_aead.so ab/pair/libcmpi_aead.so@lane_pair=1 3 > gpurun_out/r04u_pair_ab.txt 2> gpurun_out/r04u_pair_ab.err
echo AB_DONE
PMC_GROUPS=$'FETCH_SIZE\nWRITE_SIZE' PMC_OUT=gpurun_out/r04u_pmc_base WL=gcm1k timeout -k 10 200 bash tools/gpu_pmc.sh
PMC_GROUPS=$'FETCH_SIZE\nWRITE_SIZE' PMC_OUT=gpurun_out/r04u_pmc_pair WL=gcm1k AB_HOOKS=lane_pair=1 timeout -k 10 200 bash tools/gpu_pmc.sh
echo PMC_DONE
