set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=r05ao
timeout -k 10 300 python tools/sustained_ab.py ab/base/libcmpi_aead.so ab/pprio/libcmpi_aead.so 4 alltoall > gpurun_out/${R}_flow_pprio_a2a.txt 2>&1 || exit $?
timeout -k 10 400 python tools/flow_ab.py ab/base/libcmpi_aead.so ab/pprio/libcmpi_aead.so 3 > gpurun_out/${R}_flow_pprio_ab.txt 2>&1 || exit $?
echo DONE
