#!/bin/bash
# aligned-window lane stores: GCM tests, A/B (hook on/off, same build), PMC write traffic on/off
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_gcm.py tests/test_gpu_coll.py tests/test_gpu_frame.py > gpurun_out/r04j_tests.log 2>&1 || exit $?
timeout -k 10 600 python -u tools/flow_ab.py ab/new/libcmpi_aead.so@lane_aligned=0 ab/new/libcmpi_aead.so@lane_aligned=1 3 > gpurun_out/r04j_align_ab.txt 2> gpurun_out/r04j_align_ab.err || exit $?
for al in 0 1; do
  AB_HOOKS=lane_aligned=$al WL=gcm1k PMC_GROUPS="FETCH_SIZE
WRITE_SIZE" timeout -k 10 200 bash tools/gpu_pmc.sh || exit $?
  mv gpurun_out/pmc_gcm1k gpurun_out/pmc_gcm1k_al$al
done
echo ALL_DONE
