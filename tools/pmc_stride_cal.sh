set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
for st in 1040 1088 1152; do
  out=gpurun_out/cal/s$st; mkdir -p $out
  timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $out/w -o run -- python3 tools/prof_driver.py --iters 5 --out-stride $st > $out/w.log 2>&1 || exit $?
  timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $out/f -o run -- python3 tools/prof_driver.py --iters 5 --out-stride $st > $out/f.log 2>&1 || exit $?
done
echo done
