set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_gcm.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_gcm.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/t_gcm.log; exit 1; }
tail -3 gpurun_out/t_gcm.log
timeout -k 10 300 python -u tools/ab_wide.py > gpurun_out/ab_wide.log 2>&1 || { echo "ab rc=$?"; tail -20 gpurun_out/ab_wide.log; exit 1; }
grep -v '^{' gpurun_out/ab_wide.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench2.json 2>&1; echo bench rc=$?
tail -c 1500 gpurun_out/bench2.json
