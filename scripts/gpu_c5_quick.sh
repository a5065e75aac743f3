#!/bin/bash
# Overflow-fold iteration: merge GPU tests, config 5 at 64M (timing + kernel trace), then the headline
# bench without its CPU baseline / PMC passes (agent_path and config-2 numbers). Each GPU step has its own limit.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/q; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_merge.py tests/test_gpu_affinity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/q/tests.log 2>&1
rc=$?; tail -3 gpurun_out/q/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/bench_config5.py --sizes 64000000 --reps 3 > gpurun_out/q/c5.log 2>&1 || { tail -20 gpurun_out/q/c5.log; exit 1; }
grep "^n=" gpurun_out/q/c5.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/q/trace -o run -- python tools/bench_config5.py --sizes 64000000 --reps 2 > gpurun_out/q/trace.log 2>&1 || { tail -20 gpurun_out/q/trace.log; exit 1; }
if [ -n "$BENCH" ]; then
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pmc > gpurun_out/q/bench.log 2>&1 || { tail -20 gpurun_out/q/bench.log; exit 1; }
  python -c "
import json
for l in open('gpurun_out/q/bench.log'):
    if l.startswith('{'):
        d=json.loads(l); print('ms/step %.3f'%d['ms_per_step'], 'frac %.4f'%d['roofline']['frac'], 'agent_path', d.get('agent_path',{}).get('ms'), 'agent_e2e', d.get('agent_e2e',{}).get('ms'))
"
fi
