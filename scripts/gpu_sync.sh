#!/bin/bash
# Config-4 need diff: parity tests, then bench_sync (packed) with its PMC passes.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/sync; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_sync.py tests/test_gpu_scale.py -m gpu -x -q --timeout 300 --timeout-method thread -k "sync or needs or config4" > gpurun_out/sync/tests.log 2>&1
rc=$?; tail -3 gpurun_out/sync/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench_sync.py > gpurun_out/sync/bench.log 2>&1 || { tail -5 gpurun_out/sync/bench.log; exit 1; }
grep '^{' gpurun_out/sync/bench.log | cut -c1-2500
