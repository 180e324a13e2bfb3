set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/t_all.log; exit 1; }
tail -1 gpurun_out/t_all.log
timeout -k 10 400 python -u tools/ab_lib.py abtest/base/libcmpi_aead.so abtest/$1/libcmpi_aead.so > gpurun_out/ab_lib.log 2>&1; echo rc=$?
grep -v amdgpu gpurun_out/ab_lib.log | python3 -c "
import sys, json
for l in sys.stdin:
    j=json.loads(l)
    for wl, d in j.items():
        print(wl, {k:v['GiBps'] for k,v in d.items() if isinstance(v, dict)}, d.get('outputs_identical'))"
