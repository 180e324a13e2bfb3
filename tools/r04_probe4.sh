#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_framed_host.py tests/test_gpu_frame.py > gpurun_out/r04d_tests.log 2>&1 || exit $?
SCENARIOS=fresh,bench timeout -k 10 600 python -u tools/host_regress_probe.py --all > gpurun_out/r04d_host_regress.jsonl 2> gpurun_out/r04d_host_regress.err || exit $?
echo ALL_DONE
