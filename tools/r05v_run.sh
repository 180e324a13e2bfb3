set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=r05v
timeout -k 10 420 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/${R}_gpu_tests.log 2>&1 || exit $?
timeout -k 10 150 tools/msg_latency 2000 > gpurun_out/${R}_msg_latency.json 2> gpurun_out/${R}_msg_latency.err || exit $?
timeout -k 10 120 python tools/svc_timeline.py > gpurun_out/${R}_svc_timeline.jsonl 2> gpurun_out/${R}_svc_timeline.err || exit $?
echo DONE
