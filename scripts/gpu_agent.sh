#!/bin/bash
# Agent path check: the process_multiple_changes GPU tests, then the agent bench with stage times
# and a kernel trace. Each GPU step has its own limit.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/agent; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_agent_device.py tests/test_gpu_agent.py tests/test_gpu_golden_agent.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/agent/tests.log 2>&1
rc=$?; tail -15 gpurun_out/agent/tests.log; [ $rc -ne 0 ] && exit $rc
CORRO_AGENT_PROFILE=1 timeout -k 10 300 python -u tools/bench_agent.py > gpurun_out/agent/bench.log 2>&1 || { tail -20 gpurun_out/agent/bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/agent/bench.log | cut -c1-1500
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/agent/trace -o run -- python tools/bench_agent.py > gpurun_out/agent/trace.log 2>&1 || { tail -20 gpurun_out/agent/trace.log; exit 1; }
python tools/kstats.py gpurun_out/agent/trace | head -40
