#!/bin/bash
# Every GPU test, then the agent bench (agent_path + agent_e2e) with stage times.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/ta; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ta/tests.log 2>&1
rc=$?; tail -15 gpurun_out/ta/tests.log; [ $rc -ne 0 ] && exit $rc
CORRO_AGENT_PROFILE=1 timeout -k 10 300 python -u tools/bench_agent.py > gpurun_out/ta/bench.log 2>&1 || { tail -20 gpurun_out/ta/bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/ta/bench.log | cut -c1-1500
