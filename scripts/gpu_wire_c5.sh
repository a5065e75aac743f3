#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/wc; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_wire.py tests/test_gpu_agent_device.py tests/test_gpu_golden_agent.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/wc/tests.log 2>&1
rc=$?; tail -3 gpurun_out/wc/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u tools/bench_config5.py --sizes 64000000 --reps 3 --pmc > gpurun_out/wc/c5.log 2>&1 || { tail -5 gpurun_out/wc/c5.log; exit 1; }
grep -v amdgpu.ids gpurun_out/wc/c5.log | cut -c1-3000
