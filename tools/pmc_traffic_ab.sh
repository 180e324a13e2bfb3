#!/bin/bash
# HBM traffic of GCM lane-kernel variants (FETCH_SIZE / WRITE_SIZE, one counter per pass) on one
# box: VARIANTS = "form:sched ..." (cmpi_debug_set_gcm_form / cmpi_debug_set_sched).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for v in ${VARIANTS:-0:16391 1:16391}; do
  form=${v%%:*}; sched=${v##*:}
  for c in FETCH_SIZE WRITE_SIZE; do
    out=gpurun_out/pmc_ab/f${form}_s${sched}/$c
    mkdir -p "$out"
    FORM=$form SCHED=$sched timeout -k 10 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$out" -o run -- \
        python3 tools/prof_driver.py --workload "${WL:-gcm1k}" --iters 5 > "$out.log" 2>&1 || exit $?
  done
done
echo done
