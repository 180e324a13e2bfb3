set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=r05ac
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_service.py tests/test_gpu_evp_shim.py tests/test_gpu_errors.py tests/test_gpu_gcm.py > gpurun_out/${R}_svc8_tests.log 2>&1 || exit $?
CMPI_LIB=$PWD/ab/svc16/libcmpi_aead.so timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_service.py > gpurun_out/${R}_svc16_tests.log 2>&1 || exit $?
for r in 1 2; do
  for v in svc8 svc16; do
    LD_LIBRARY_PATH=$PWD/ab/$v timeout -k 10 150 tools/msg_latency 1000 > gpurun_out/${R}_msg_latency_${v}_$r.json 2> gpurun_out/${R}_msg_latency_${v}_$r.err || exit $?
  done
done
echo DONE
