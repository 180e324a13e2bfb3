set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=r05av
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_${R}_a2a -o run -- python3 tools/prof_driver.py --workload alltoall --iters 2000 > gpurun_out/${R}_prof.log 2>&1 || exit $?
echo DONE
