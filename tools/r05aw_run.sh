set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=r05aw
for w in 0.5 2.0 0.5 2.0 0.5 2.0; do
  CMPI_BENCH_WARMUP_S=$w timeout -k 10 200 python bench.py --no-extras >> gpurun_out/${R}_warmup_sweep.jsonl 2>> gpurun_out/${R}_warmup_sweep.err || exit $?
done
echo DONE
