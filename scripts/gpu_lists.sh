#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/li; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_merge.py tests/test_gpu_agent_device.py tests/test_gpu_golden_agent.py tests/test_gpu_agent.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/li/tests.log 2>&1
rc=$?; tail -3 gpurun_out/li/tests.log; [ $rc -ne 0 ] && exit $rc
for v in lists0 default; do
  L=""; [ $v != default ] && L=tools/_variants/libcorro_$v.so
  CORRO_HIP_LIB=$L CORRO_AGENT_REPS=5 timeout -k 10 300 python -u tools/bench_agent.py > gpurun_out/li/b_$v.log 2>&1 || { tail -5 gpurun_out/li/b_$v.log; exit 1; }
  echo "$v $(grep '^{' gpurun_out/li/b_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["agent_path"]["ms"],3), round(d["agent_path"]["merge_ms"],3), round(d["agent_e2e"]["ms"],3))')"
done
