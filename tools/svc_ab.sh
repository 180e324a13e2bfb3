#!/bin/bash
# Interleaved A/B of the single-message latency (tools/msg_latency) between two engine builds placed
# as ab/base/libcmpi_aead.so and ab/new/libcmpi_aead.so (msg_latency's RUNPATH yields to
# LD_LIBRARY_PATH), three rounds, then the service / EVP / 600 tests against the in-tree build.
# Run on a GPU box from the repo root: bash tools/svc_ab.sh; results in gpurun_out/ml_{base,new}_N.json.
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
  for v in base new; do
    LD_LIBRARY_PATH=ab/$v timeout -k 10 120 tools/msg_latency 2000 > gpurun_out/ml_${v}_$i.json 2> gpurun_out/ml_${v}_$i.err || exit $?
  done
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_service.py tests/test_gpu_evp_shim.py tests/test_gpu_p2p.py > gpurun_out/svc_tests.log 2>&1
