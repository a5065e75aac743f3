#!/bin/bash
# Round check: smoke, every GPU test, bench (with CPU baseline), rocprofv3 kernel stats of the bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; tail -n 3 "gpurun_out/$name.log" | cut -c1-400; [ $rc -ne 0 ] && { echo "FAIL $name rc=$rc"; exit $rc; }; return 0; }
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step bench 600 python -u bench.py
step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline
python tools/kstats.py gpurun_out/prof | head -12
