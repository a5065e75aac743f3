#!/bin/bash
# Every GPU test, the bench line, config 5 with its PMC traffic passes. Each GPU step has its own limit.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/f3; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/f3/tests.log 2>&1
rc=$?; tail -4 gpurun_out/f3/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/f3/bench.log 2>&1 || { tail -5 gpurun_out/f3/bench.log; exit 1; }
grep '^{' gpurun_out/f3/bench.log | cut -c1-600
timeout -k 10 700 python -u tools/bench_config5.py --sizes 64000000 --reps 3 --pmc > gpurun_out/f3/c5.log 2>&1 || { tail -5 gpurun_out/f3/c5.log; exit 1; }
grep -v amdgpu.ids gpurun_out/f3/c5.log | cut -c1-2500
