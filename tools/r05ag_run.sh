set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=r05ag
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_ctr_ecb_ocb.py tests/test_gpu_ctrmode.py tests/test_gpu_errors.py > gpurun_out/${R}_ctr_tests.log 2>&1 || exit $?
timeout -k 10 200 python tools/ctr_hybrid_sweep.py 0 50 100 150 200 0 > gpurun_out/${R}_ctr_hybrid_sweep.jsonl 2>&1 || exit $?
timeout -k 10 450 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/${R}_gpu_tests.log 2>&1 || exit $?
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${R}_smoke.log 2>&1 || exit $?
timeout -k 10 420 python bench.py > gpurun_out/${R}_bench.json 2> gpurun_out/${R}_bench.err || exit $?
echo DONE
