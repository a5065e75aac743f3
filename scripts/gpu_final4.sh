#!/bin/bash
# Round-3 check after the overflow-fold work. PART=a: smoke + every GPU test; PART=b: bench line,
# kernel trace of the bench, config 5 with PMC traffic, agent bench. Each GPU step has its own limit;
# a failure ends the script.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/fin4; export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/fin4/$name.log" 2>&1; local rc=$?; tail -n 2 "gpurun_out/fin4/$name.log" | cut -c1-300; [ $rc -ne 0 ] && { echo "FAIL $name rc=$rc"; exit $rc; }; return 0; }
if [ "$PART" = a ]; then
  step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
  step tests 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
else
  step bench 600 python -u bench.py
  step prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fin4/prof -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-pmc
  step c5 500 python -u tools/bench_config5.py --sizes 64000000 --reps 3 --pmc
  CORRO_AGENT_PROFILE=1 step agent 300 python -u tools/bench_agent.py
fi
echo "=== done"
