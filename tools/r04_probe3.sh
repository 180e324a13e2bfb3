#!/bin/bash
# Round-4 GPU pass 3: framed host tests (direct + DMA request forms), service / EVP tests, host-path probe
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_framed_host.py tests/test_gpu_async.py tests/test_gpu_service.py tests/test_gpu_evp_shim.py > gpurun_out/r04c_tests.log 2>&1 || exit $?
timeout -k 10 900 python -u tools/host_regress_probe.py --all > gpurun_out/r04c_host_regress.jsonl 2> gpurun_out/r04c_host_regress.err || exit $?
echo ALL_DONE
