#!/bin/bash
# Round-end GPU pass on the committed build (run through gpurun from the repo root): the whole -m gpu
# suite, smoke(), the default bench, the single-message latency table, then (PROF=1) the bench under
# rocprofv3 --kernel-trace --stats: the default command, and the headline alone (--no-extras), whose
# --stats average of the dominant kernel is the one the line's roofline uses.  Every step under its
# own time limit; the first failure ends the pass.  PMC=1 adds the config-2 counter passes
# (tools/gpu_pmc.sh).  Results in gpurun_out/${R}_*.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${ROUND:-r06}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/${R}_gpu_tests.log 2>&1 || exit $?
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${R}_smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py > gpurun_out/${R}_bench.json 2> gpurun_out/${R}_bench.err || exit $?
timeout -k 10 120 tools/msg_latency 2000 > gpurun_out/${R}_msg_latency.json 2> gpurun_out/${R}_msg_latency.err || exit $?
if [ -n "$PROF" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${R}_headline -o run -- \
      python3 bench.py --no-extras > gpurun_out/${R}_headline_under_rocprof.json 2> gpurun_out/${R}_headline_under_rocprof.err || exit $?
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${R}_bench -o run -- \
      python3 bench.py > gpurun_out/${R}_bench_under_rocprof.json 2> gpurun_out/${R}_bench_under_rocprof.err || exit $?
fi
if [ -n "$PMC" ]; then  # counters of the config-2 seal / open (summarise here: LAST=5 tools/pmc_summarize.py)
  WL=gcm1k PMC_OUT=gpurun_out/${R}_pmc_gcm1k timeout -k 10 400 bash tools/gpu_pmc.sh || exit $?
fi
echo VAL_DONE
