#!/bin/bash
# Round-3 check: smoke, every GPU test, bench line, kernel trace of the bench, config 4 / config 5 /
# agent benches. Each GPU step has its own limit; a failure ends the script.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/fin; export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/fin/$name.log" 2>&1; local rc=$?; tail -n 2 "gpurun_out/fin/$name.log" | cut -c1-300; [ $rc -ne 0 ] && { echo "FAIL $name rc=$rc"; exit $rc; }; return 0; }
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step bench 600 python -u bench.py
step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fin/prof -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline
step sync 500 python -u bench_sync.py
step c5 700 python -u tools/bench_config5.py --sizes 64000000 --reps 3 --pmc
CORRO_AGENT_PROFILE=1 step agent 300 python -u tools/bench_agent.py
echo "=== done"
