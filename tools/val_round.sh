set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/gpu_tests.log 2>&1 || exit $?
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
timeout -k 10 60 tools/probe/doorbell_probe 2000 > gpurun_out/doorbell.json 2> gpurun_out/doorbell.err || exit $?
for i in 1 2; do
  for v in host device; do
    CMPI_SERVICE_RING=$v timeout -k 10 120 tools/msg_latency 2000 > gpurun_out/ml_${v}_$i.json 2> gpurun_out/ml_${v}_$i.err || exit $?
  done
done
