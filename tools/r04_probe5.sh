#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/host_pipe_sweep.py > gpurun_out/r04e_host_sweep.json 2> gpurun_out/r04e_host_sweep.err || exit $?
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r04e_gpu_tests.log 2>&1 || exit $?
timeout -k 10 200 tools/msg_latency 2000 > gpurun_out/r04e_msg_latency.json 2> gpurun_out/r04e_msg_latency.err || exit $?
echo ALL_DONE
