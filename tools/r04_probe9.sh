#!/bin/bash
# Round 4: the paired-store lane kernel at sustained clocks (tools/sustained_ab.py) on configs 2
# and the 4 KiB workload, and a longer burst A/B on the lane shapes.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/sustained_ab.py ab/pair/libcmpi_aead.so ab/pair/libcmpi_aead.so@lane_pair=1 4 gcm1k > gpurun_out/r04v_sustained_gcm1k.txt 2>&1
echo S1
timeout -k 10 300 python -u tools/sustained_ab.py ab/pair/libcmpi_aead.so ab/pair/libcmpi_aead.so@lane_pair=1 3 gcm4k > gpurun_out/r04v_sustained_gcm4k.txt 2>&1
echo S2
AB_SHAPES=65536x1000,65536x1024,65536x4096,2048x200 timeout -k 10 300 python -u tools/flow_ab.py ab/pair/libcmpi_aead.so ab/pair/libcmpi_aead.so@lane_pair=1 5 > gpurun_out/r04v_pair_ab.txt 2>&1
echo AB
