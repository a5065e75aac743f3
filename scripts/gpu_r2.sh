#!/bin/bash
# Round-2 GPU check: GPU tests, the N=1 bench (live PMC traffic + CPU baseline), a 2-rank gloo
# rehearsal of the N>1 strong-scaling bench on this one GPU, and a kernel trace of the N=1 bench.
# Each GPU step has its own limit; a failure ends the script.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r2; export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/r2/$name.log" 2>&1; local rc=$?; tail -n 4 "gpurun_out/r2/$name.log" | cut -c1-600; if [ $rc -ne 0 ]; then echo "FAIL $name rc=$rc"; exit $rc; fi; return 0; }
[ -z "$SKIP_TESTS" ] && step tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${TESTS:-}
[ -z "$SKIP_SMOKE" ] && step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
[ -z "$SKIP_BENCH" ] && step bench 600 python -u bench.py
[ -n "$MULTI" ] && step bench_gloo2 600 env CORRO_BENCH_BACKEND=gloo python -u bench.py --gpus 2 --changes ${MULTI_CHANGES:-67108864} --steps 2 --warmup 1
[ -n "$TRACE" ] && step trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2/trace -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-pmc
[ -n "$TRACE" ] && python tools/kstats.py gpurun_out/r2/trace | head -14
echo "=== done"
