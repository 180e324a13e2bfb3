#!/bin/bash
# Build libcmpi_aead.so of git revision REV into abtest/NAME/ (for tools/ab_lib.py A/B runs).
# Usage: tools/ab_build.sh REV NAME      (REV "WORK" = the current working tree)
set -eu
cd "$(dirname "$0")/.."
rev=$1 name=$2
mkdir -p "abtest/$name"
if [ "$rev" = WORK ]; then
  make -C cryptmpi_2022_amd -s
  cp cryptmpi_2022_amd/libcmpi_aead.so "abtest/$name/"
else
  wt=$(mktemp -d /tmp/abwt.XXXX)
  git worktree add -q --detach "$wt" "$rev"
  make -C "$wt/cryptmpi_2022_amd" -s libcmpi_aead.so
  cp "$wt/cryptmpi_2022_amd/libcmpi_aead.so" "abtest/$name/"
  git worktree remove --force "$wt"
fi
echo "abtest/$name/libcmpi_aead.so"
