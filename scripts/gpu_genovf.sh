#!/bin/bash
# Config 5: general buckets above N records routed to the device-wide fold (CORRO_GEN_OVF_MIN A/B).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/go; export TMPDIR=/tmp
for n in 4294967295 1024 512 256 0; do
  CORRO_GEN_OVF_MIN=$n timeout -k 10 200 python -u tools/bench_config5.py --sizes 64000000 --reps 3 > gpurun_out/go/c5_$n.log 2>&1 || { tail -20 gpurun_out/go/c5_$n.log; exit 1; }
  echo "GEN_OVF_MIN=$n $(grep '^n=' gpurun_out/go/c5_$n.log)"
done
CORRO_GEN_OVF_MIN=256 timeout -k 10 400 python -u -m pytest tests/test_gpu_merge.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/go/tests.log 2>&1
rc=$?; tail -3 gpurun_out/go/tests.log; exit $rc
