#!/bin/bash
# One GPU-box pass of the round's checks (run through gpurun from the repo root): the resident
# service, EVP shim and 2-process 600 tests, the per-message latency breakdown, the whole -m gpu
# suite, the default bench.  Every step under its own time limit; the first failure ends the pass.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_service.py tests/test_gpu_evp_shim.py tests/test_gpu_p2p.py > gpurun_out/svc_tests.log 2>&1 || exit $?
timeout -k 10 120 tools/msg_latency 2000 > gpurun_out/msg_latency.json 2> gpurun_out/msg_latency.err || exit $?
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
timeout -k 10 150 python tools/framed_rates.py > gpurun_out/framed_rates.json 2> gpurun_out/framed_rates.err || exit $?
