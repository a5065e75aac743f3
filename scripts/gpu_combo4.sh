#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/c4; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_agent_device.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/c4/tests.log 2>&1
rc=$?; tail -4 gpurun_out/c4/tests.log; [ $rc -ne 0 ] && exit $rc
bash scripts/gpu_sync_diag.sh
