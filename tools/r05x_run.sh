set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=r05x
timeout -k 10 420 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/${R}_gpu_tests.log 2>&1 || exit $?
timeout -k 10 150 tools/msg_latency 2000 > gpurun_out/${R}_msg_latency.json 2> gpurun_out/${R}_msg_latency.err || exit $?
timeout -k 10 120 python tools/svc_timeline.py > gpurun_out/${R}_svc_timeline.jsonl 2> gpurun_out/${R}_svc_timeline.err || exit $?
timeout -k 10 200 python tools/sustained_ab.py ab/base/libcmpi_aead.so ab/sep/libcmpi_aead.so 3 alltoall > gpurun_out/${R}_alltoall_ab.txt 2>&1 || exit $?
echo DONE
