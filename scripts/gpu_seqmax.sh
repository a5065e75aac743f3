#!/bin/bash
# Config 5: short overflow rows (<= N sorted records) folded sequentially in the walk (CORRO_OVF_SEQ_MAX A/B),
# then parity with the routing on. Each GPU step has its own limit.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/sq; export TMPDIR=/tmp
for n in 0 4 16 64; do
  CORRO_OVF_SEQ_MAX=$n timeout -k 10 200 python -u tools/bench_config5.py --sizes 64000000 --reps 3 > gpurun_out/sq/c5_$n.log 2>&1 || { tail -20 gpurun_out/sq/c5_$n.log; exit 1; }
  echo "SEQ_MAX=$n $(grep '^n=' gpurun_out/sq/c5_$n.log)"
done
CORRO_OVF_SEQ_MAX=16 timeout -k 10 400 python -u -m pytest tests/test_gpu_merge.py tests/test_gpu_ovf_reduce.py tests/test_gpu_long.py tests/test_gpu_affinity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/sq/tests.log 2>&1
rc=$?; tail -3 gpurun_out/sq/tests.log; exit $rc
