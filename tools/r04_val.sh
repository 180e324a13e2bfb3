#!/bin/bash
# Round-4 validation + profile pass on one box: GPU suite, smoke, the default bench under
# rocprofv3 --kernel-trace --stats (csv) after a plain run of it, msg_latency.  Each step time-limited; first failure ends it.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${ROUND:-r04m}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/${R}_gpu_tests.log 2>&1 || exit $?
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${R}_smoke.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py > gpurun_out/${R}_bench.json 2> gpurun_out/${R}_bench.err || exit $?
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${R}_bench -o run -- \
    python3 bench.py > gpurun_out/${R}_bench_under_rocprof.json 2> gpurun_out/${R}_bench_under_rocprof.err || exit $?
timeout -k 10 300 tools/msg_latency 2000 > gpurun_out/${R}_msg_latency.json 2> gpurun_out/${R}_msg_latency.err || exit $?
echo VAL_DONE
