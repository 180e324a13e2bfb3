set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=r05z
timeout -k 10 200 python tools/sustained_ab.py ab/base/libcmpi_aead.so ab/c0abl/libcmpi_aead.so 3 alltoall > gpurun_out/${R}_chunk0_ablation.txt 2>&1 || exit $?
timeout -k 10 150 tools/msg_latency 2000 > gpurun_out/${R}_msg_latency.json 2> gpurun_out/${R}_msg_latency.err || exit $?
WL=gcm1k PMC_OUT=gpurun_out/${R}_pmc_gcm1k timeout -k 10 400 bash tools/gpu_pmc.sh || exit $?
WL=alltoall PMC_OUT=gpurun_out/${R}_pmc_alltoall timeout -k 10 400 bash tools/gpu_pmc.sh || exit $?
echo DONE
