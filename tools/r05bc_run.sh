set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=r05bc
CMPI_LIB=$PWD/ab/cwave/libcmpi_aead.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_gcm.py tests/test_gpu_coll.py > gpurun_out/${R}_cwave_tests.log 2>&1 || exit $?
timeout -k 10 300 python tools/sustained_ab.py ab/base/libcmpi_aead.so ab/cwave/libcmpi_aead.so 5 alltoall > gpurun_out/${R}_cwave_a2a.txt 2>&1 || exit $?
AB_SHAPES="8x1MiB,1x8MiB,32x256KiB,8x(1MiB-5),3x100000" timeout -k 10 300 python tools/flow_ab.py ab/base/libcmpi_aead.so ab/cwave/libcmpi_aead.so 3 > gpurun_out/${R}_cwave_ab.txt 2>&1 || exit $?
echo DONE
