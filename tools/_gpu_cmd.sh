set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { echo "pytest rc=$?"; tail -40 gpurun_out/t_all.log; exit 1; }
tail -1 gpurun_out/t_all.log
timeout -k 10 300 python -u tools/ab_602.py > gpurun_out/ab_602.log 2>&1; echo rc=$?
grep -v amdgpu gpurun_out/ab_602.log | grep -v '^{'
