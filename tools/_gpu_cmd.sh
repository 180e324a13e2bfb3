set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "host or evp or frame or 600 or 602" > gpurun_out/t_host.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/t_host.log; exit 1; }
tail -1 gpurun_out/t_host.log
for i in 1 2; do timeout -k 10 300 python -c "
import bench, json
print(json.dumps(bench.host_path_rate(0)))" 2>&1 | grep -v amdgpu.ids; done
