set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/t_all.log; exit 1; }
tail -1 gpurun_out/t_all.log
timeout -k 10 300 python -u tools/ab_wide.py > gpurun_out/ab_wide.log 2>&1; echo rc=$?
grep -v '^{' gpurun_out/ab_wide.log | grep -v amdgpu | grep "alltoall\|auto\|lanes"
