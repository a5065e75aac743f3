#!/bin/bash
# Overflow row reduction: parity (merge + affinity GPU tests, config 5 at 64M without impacts), then
# config 5 with the reduction on and off, and a kernel trace with it on. Each GPU step has its own limit.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/red; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_merge.py tests/test_gpu_affinity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/red/tests.log 2>&1
rc=$?; tail -5 gpurun_out/red/tests.log; [ $rc -ne 0 ] && exit $rc
CORRO_HIP_OVF_DEBUG=1 timeout -k 10 300 python -u tools/bench_config5.py --sizes 64000000 --reps 3 > gpurun_out/red/on.log 2>&1 || { tail -20 gpurun_out/red/on.log; exit 1; }
grep -v amdgpu.ids gpurun_out/red/on.log | sort | uniq -c | sort -rn | head -8 | cut -c1-400
CORRO_OVF_REDUCE=0 timeout -k 10 300 python -u tools/bench_config5.py --sizes 64000000 --reps 3 > gpurun_out/red/off.log 2>&1 || { tail -20 gpurun_out/red/off.log; exit 1; }
grep "^n=" gpurun_out/red/off.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/red/trace -o run -- python tools/bench_config5.py --sizes 64000000 --reps 2 > gpurun_out/red/trace.log 2>&1 || { tail -20 gpurun_out/red/trace.log; exit 1; }
f=$(find gpurun_out/red/trace -name '*kernel_stats.csv' | head -1); cut -d, -f1-5 "$f" | head -32
timeout -k 10 900 python -u -m pytest "tests/test_gpu_scale.py::test_config5_64m_two_batch_fold_vs_sharded_oracle[no_impacts]" -m gpu -x -q -s --timeout 880 --timeout-method thread > gpurun_out/red/scale.log 2>&1
rc=$?; tail -8 gpurun_out/red/scale.log; exit $rc
