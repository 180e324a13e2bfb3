#!/bin/bash
# Round 4: the flow kernel with the length block out of the step slots — GCM / service / framed
# parity, then the A/B on the flow shapes against the previous build (ab/pair).
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_gcm.py tests/test_gpu_service.py tests/test_gpu_framed_host.py tests/test_gpu_frame.py tests/test_gpu_evp_shim.py > gpurun_out/r04za_tests.log 2>&1
echo TESTS
AB_SHAPES=8x1MiB,1x64KiB,3x100000,1x8MiB,32x256KiB,8x\(1MiB-5\),1x1000,64x1000,2048x1000,16x100,1x100,2048x600,256x260 timeout -k 10 400 python -u tools/flow_ab.py ab/pair/libcmpi_aead.so ab/nolen/libcmpi_aead.so 3 > gpurun_out/r04za_nolen_ab.txt 2> gpurun_out/r04za_nolen_ab.err
echo AB
timeout -k 10 300 tools/msg_latency 500 > gpurun_out/r04za_msg_latency.json 2> gpurun_out/r04za_msg_latency.err
echo LAT
