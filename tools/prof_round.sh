set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_gcm1k -o run -- python3 bench.py --no-extras --no-cpu-baseline > gpurun_out/bench_under_rocprof.log 2>&1
WL=gcm1k timeout -k 10 400 bash tools/gpu_pmc.sh
echo PROF_DONE
