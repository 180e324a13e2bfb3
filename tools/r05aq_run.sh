set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=r05aq
CMPI_LIB=$PWD/ab/late/libcmpi_aead.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_gcm.py tests/test_gpu_framed_host.py > gpurun_out/${R}_late_tests.log 2>&1 || exit $?
timeout -k 10 300 python tools/sustained_ab.py ab/base/libcmpi_aead.so ab/tagpf/libcmpi_aead.so 4 alltoall > gpurun_out/${R}_tagpf_a2a.txt 2>&1 || exit $?
timeout -k 10 300 python tools/sustained_ab.py ab/tagpf/libcmpi_aead.so ab/late/libcmpi_aead.so 4 alltoall > gpurun_out/${R}_late_a2a.txt 2>&1 || exit $?
timeout -k 10 400 python tools/flow_ab.py ab/tagpf/libcmpi_aead.so ab/late/libcmpi_aead.so 3 > gpurun_out/${R}_late_ab.txt 2>&1 || exit $?
echo DONE
