set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=r05t
timeout -k 10 420 python bench.py > gpurun_out/${R}_bench.json 2> gpurun_out/${R}_bench.err || exit $?
timeout -k 10 150 tools/msg_latency 2000 > gpurun_out/${R}_msg_latency.json 2> gpurun_out/${R}_msg_latency.err || exit $?
timeout -k 10 400 python tools/sustained_ab.py ab/base/libcmpi_aead.so ab/p2/libcmpi_aead.so ab/p4/libcmpi_aead.so ab/p8/libcmpi_aead.so 3 > gpurun_out/${R}_prio_ab.txt 2>&1 || exit $?
for v in base p4; do
  CMPI_LIB=$PWD/ab/$v/libcmpi_aead.so PMC_OUT=gpurun_out/${R}_pmc_$v PMC_GROUPS="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES" timeout -k 10 200 bash tools/gpu_pmc.sh || exit $?
done
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${R}_bench -o run -- python3 bench.py > gpurun_out/${R}_bench_under_rocprof.json 2> gpurun_out/${R}_bench_under_rocprof.err || exit $?
echo DONE
