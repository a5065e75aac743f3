#!/bin/bash
# One GPU session: smoke, GPU parity tests, bench, rocprofv3 kernel-trace summary.
# Each GPU step has its own time limit; a crash/timeout/abort ends the script (no retries).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS="${STEPS:-smoke tests bench prof}"
run() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "ABORT after $name"; exit $rc; fi
  return 0
}
for s in $STEPS; do
  case $s in
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) run tests 600 python -m pytest tests -m gpu -q -x ;;
    bench) run bench 600 python bench.py --steps 10 --warmup 3 ;;
    prof)  run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline ;;
  esac
done
echo "=== done"
