#!/bin/bash
# Round-4 first GPU pass: the new 8-rank config-5 test and the high-bit host address test, the
# hardware-queue probe (tools/queue_probe.py), then PMC passes of the config-5 / OCB / CTR kernels.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_alltoall8.py "tests/test_gpu_service.py::test_high_bit_host_addresses" \
  "tests/test_gpu_coll.py::test_bench_alltoall_e2e_one_rank" > gpurun_out/r04a_tests.log 2>&1 || exit $?
timeout -k 10 500 python -u tools/queue_probe.py --all > gpurun_out/r04a_queue_probe.jsonl 2> gpurun_out/r04a_queue_probe.err || exit $?
for wl in alltoall ocb1m ctr1g; do
  WL=$wl timeout -k 10 300 bash tools/gpu_pmc.sh || exit $?
done
echo ALL_DONE
