#!/bin/bash
# Config-4 need diff: buffered-emission variants (NEED_NB = 0 old form, 2, 3, 4 default), parity tests first.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/sync; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_sync.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/sync/tests.log 2>&1
rc=$?; tail -3 gpurun_out/sync/tests.log; [ $rc -ne 0 ] && exit $rc
for v in nb0 nb2 nb3; do
  CORRO_HIP_LIB=tools/_variants/libcorro_$v.so timeout -k 10 200 python -u bench_sync.py --no-pmc --cpu-sample 1000 > gpurun_out/sync/b_$v.log 2>&1 || { tail -5 gpurun_out/sync/b_$v.log; exit 1; }
  echo "$v $(grep '^{' gpurun_out/sync/b_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("roofline",{}).get("frac"))')"
done
timeout -k 10 400 python -u bench_sync.py --cpu-sample 1000 > gpurun_out/sync/b_nb4.log 2>&1 || { tail -5 gpurun_out/sync/b_nb4.log; exit 1; }
grep '^{' gpurun_out/sync/b_nb4.log | cut -c1-1500
