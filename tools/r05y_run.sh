set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=r05y
timeout -k 10 420 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/${R}_gpu_tests.log 2>&1 || exit $?
timeout -k 10 150 tools/msg_latency 2000 > gpurun_out/${R}_msg_latency.json 2> gpurun_out/${R}_msg_latency.err || exit $?
timeout -k 10 200 python -c "import json,bench; print(json.dumps(bench.host602_rate(0)))" > gpurun_out/${R}_host602.json 2> gpurun_out/${R}_host602.err || exit $?
numactl -H > gpurun_out/${R}_numa.txt 2>&1 || true
echo DONE
