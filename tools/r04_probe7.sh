#!/bin/bash
# device-made chunk weights for 602 sub-key contexts + DPP/permlane lane exchanges (+ transpose-
# free lane tree in new2): tests (in-tree = new2), 602 rates, flow/lane shape A/B, msg latency
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_frame.py tests/test_gpu_framed_host.py tests/test_gpu_gcm.py tests/test_gpu_evp_shim.py tests/test_gpu_service.py tests/test_gpu_ctr_ecb_ocb.py tests/test_gpu_coll.py > gpurun_out/r04o_tests.log 2>&1 || exit $?
for b in base new2 base new2; do
  CMPI_LIB=ab/$b/libcmpi_aead.so timeout -k 10 200 python -u tools/framed_rates.py >> gpurun_out/r04o_framed_$b.jsonl 2>> gpurun_out/r04o_framed.err || exit $?
done
timeout -k 10 600 python -u tools/flow_ab.py ab/base/libcmpi_aead.so ab/new/libcmpi_aead.so 3 > gpurun_out/r04o_flow_ab.txt 2> gpurun_out/r04o_flow_ab.err || exit $?
timeout -k 10 600 python -u tools/flow_ab.py ab/new/libcmpi_aead.so ab/new2/libcmpi_aead.so 3 > gpurun_out/r04o_flow_ab2.txt 2> gpurun_out/r04o_flow_ab2.err || exit $?
timeout -k 10 300 tools/msg_latency 1000 > gpurun_out/r04o_msg_latency.json 2> gpurun_out/r04o_msg_latency.err || exit $?
echo ALL_DONE
