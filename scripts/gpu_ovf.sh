#!/bin/bash
# Overflow-path check: merge parity tests, then the config-5 probe with overflow stats.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/c5; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_merge.py tests/test_gpu_agent.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/c5/tests.log 2>&1
rc=$?; tail -5 gpurun_out/c5/tests.log; [ $rc -ne 0 ] && exit $rc
CORRO_HIP_OVF_DEBUG=1 timeout -k 10 300 python -u tools/bench_config5.py --sizes ${SIZES:-16000000,64000000} --reps 3 > gpurun_out/c5/probe.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/c5/probe.log | sort | uniq -c | sort -rn | head -12; exit $rc
