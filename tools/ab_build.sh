#!/bin/bash
# Reproducible A/B builds of the engine (the recipe every "measured, taken / not taken" entry in
# DESIGN.md uses).  Builds ab/<name>/libcmpi_aead.so from a named git revision (or the working
# tree) with optional extra compiler flags (e.g. -DCMPI_LDS_BATCH=1 for a compile-time variant):
#
#   tools/ab_build.sh <name> <git-rev|WORKTREE> [extra hipcc flags...]
#
# then compare on a GPU box, interleaved, at sustained clocks:
#
#   python tools/sustained_ab.py ab/base/libcmpi_aead.so ab/new/libcmpi_aead.so [rounds] [workload]
#   python tools/flow_ab.py      ab/base/libcmpi_aead.so ab/new/libcmpi_aead.so [rounds]
#   LD_LIBRARY_PATH=ab/<name> tools/msg_latency 2000          (single-message latency)
#
# ab/ is git-ignored and travels to the GPU box with the tree (build here, on the CPU).
set -euo pipefail
[ $# -ge 2 ] || { sed -n 2,14p "$0"; exit 2; }
name=$1 rev=$2
shift 2
root=$(cd "$(dirname "$0")/.." && pwd)
out=$root/ab/$name
mkdir -p "$out"
if [ "$rev" = WORKTREE ]; then
  src=$root
else
  src=$(mktemp -d)
  trap 'rm -rf "$src"' EXIT
  git -C "$root" archive "$rev" cryptmpi_2022_amd/csrc include | tar -x -C "$src"
fi
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -munsafe-fp-atomics \
  "$@" -shared -o "$out/libcmpi_aead.so" "$src/cryptmpi_2022_amd/csrc/cmpi_aead.hip"
echo "$out/libcmpi_aead.so ($rev $*)"
