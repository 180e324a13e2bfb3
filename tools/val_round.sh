# Round-end GPU pass on the committed build (run through gpurun from the repo root): the whole -m gpu
# suite, smoke(), the default bench and the single-message latency table.  Every step under its own
# time limit; the first failure ends the pass.  Results in gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/gpu_tests.log 2>&1 || exit $?
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
timeout -k 10 120 tools/msg_latency 2000 > gpurun_out/msg_latency.json 2> gpurun_out/msg_latency.err || exit $?
