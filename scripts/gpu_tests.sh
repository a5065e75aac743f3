#!/bin/bash
# GPU parity tests (optionally a subset: TESTS="tests/test_gpu_extract.py"), one pytest process.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR" gpurun_out/tests.log | tail -${TAILN:-15}; tail -3 gpurun_out/tests.log; exit $rc
