set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=r05am
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_ctr_ecb_ocb.py -k "ctr" > gpurun_out/${R}_ctr_tests.log 2>&1 || exit $?
timeout -k 10 200 python tools/ctr_hybrid_sweep.py 0 1000 100 150 200 250 0 > gpurun_out/${R}_ctr_hybrid_sweep.jsonl 2>&1 || exit $?
echo DONE
