#!/bin/bash
# PMC passes (one counter group per pass, --kernel-trace only, never with sys/runtime traces).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=${PMC_OUT:-gpurun_out/pmc_${WL:-gcm1k}}
mkdir -p "$out"
export TMPDIR=/tmp
WL=${WL:-gcm1k}
rocprofv3 -L > "$out/counters_list.txt" 2>&1 || true
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  echo "[$(date +%T)] pass $i: $grp" >> "$out/steps.log"
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$out/p$i" -o run -- \
      python3 tools/prof_driver.py --workload "$WL" --iters 5 > "$out/p$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc" >> "$out/steps.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done <<GROUPS
${PMC_GROUPS:-FETCH_SIZE
WRITE_SIZE
SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES
SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT
GRBM_GUI_ACTIVE SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM_RD}
GROUPS
echo done >> "$out/steps.log"
