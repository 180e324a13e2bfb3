#!/bin/bash
# One GPU-box session: smoke -> gpu parity tests -> bench -> rocprofv3 kernel stats.
# Stops at the first step that crashes, times out or faults (exit codes other than 0/1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out
mkdir -p "$out"
: > "$out/steps.log"
export TMPDIR=/tmp
step() {  # step NAME SECONDS LOGFILE CMD...
  local name=$1 secs=$2 log=$3
  shift 3
  echo "[$(date +%T)] start $name" >> "$out/steps.log"
  timeout -k 10 "$secs" "$@" > "$log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" >> "$out/steps.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "stopping after $name (rc=$rc)" >> "$out/steps.log"
    exit $rc
  fi
}
WHAT=${1:-all}
if [[ $WHAT == all || $WHAT == *smoke* ]]; then
  step smoke 240 "$out/smoke.log" python -c "import __graft_entry__ as g; g.smoke()"
fi
if [[ $WHAT == all || $WHAT == *test* ]]; then
  step pytest_gpu 900 "$out/pytest_gpu.log" python -u -m pytest tests -m gpu -q -rf --timeout 180 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"}
fi
if [[ $WHAT == all || $WHAT == *bench* ]]; then
  step bench 600 "$out/bench.json" python bench.py ${BENCH_ARGS:-}
fi
if [[ $WHAT == all || $WHAT == *prof* ]]; then
  step rocprof 600 "$out/rocprof.log" rocprofv3 --kernel-trace --stats -d "$out/prof" -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-extras --steps 20 --warmup 3 ${PROF_ARGS:-}
fi
echo "done" >> "$out/steps.log"
