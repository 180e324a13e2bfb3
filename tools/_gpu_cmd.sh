set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/ab_lib.py abtest/base/libcmpi_aead.so abtest/fold/libcmpi_aead.so > gpurun_out/ab_lib.log 2>&1; echo rc=$?
grep -v amdgpu gpurun_out/ab_lib.log | tail -40
