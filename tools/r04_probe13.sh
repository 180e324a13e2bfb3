#!/bin/bash
# Round 4: kernel durations of two builds on the same shapes (rocprofv3 --kernel-trace --stats):
# is a slowdown between builds in the kernels or on the host?
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for b in pair nolen; do
  CMPI_LIB=$PWD/ab/$b/libcmpi_aead.so AB_SHAPES=8x1MiB,16x100 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04za_prof_$b -o run -- python3 tools/flow_ab.py --child ab/$b/libcmpi_aead.so > gpurun_out/r04za_prof_$b.log 2>&1
  echo $b
done
