set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=r05ah
timeout -k 10 300 python tools/sustained_ab.py ab/base/libcmpi_aead.so ab/late/libcmpi_aead.so 4 > gpurun_out/${R}_prio_late_ab.txt 2>&1 || exit $?
CMPI_LIB=$PWD/ab/late/libcmpi_aead.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_gcm.py -k "batch or config2 or lane" > gpurun_out/${R}_late_tests.log 2>&1 || exit $?
timeout -k 10 120 python tools/ctr_hybrid_sweep.py 0 1000 0 > gpurun_out/${R}_ctr_bs_alone.jsonl 2>&1 || exit $?
echo DONE
