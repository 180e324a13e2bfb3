#!/bin/bash
# One GPU-box pass of the round's checks (run through gpurun from the repo root): the resident
# service + EVP shim tests, the per-message latency breakdown, the whole -m gpu suite, the default
# bench.  Every step under its own time limit; the first failure ends the pass.
set -o pipefail
mkdir -p gpurun_out
for v in v1 sys0 sys1; do
  LD_LIBRARY_PATH=tools/svc_var/$v timeout -k 10 120 tools/msg_latency 1000 > gpurun_out/msg_latency_$v.json 2> gpurun_out/msg_latency_$v.err || exit $?
done
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/gpu_tests.log 2>&1 || exit $?
