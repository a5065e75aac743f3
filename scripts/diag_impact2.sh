#!/bin/bash
# Phase clocks of the packed impact body and of the plain body (diagnostic builds, results not valid).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/diag2
DIAG_IMPACT=1 timeout -k 10 300 python -u tools/diag_merge.py tools/_variants/libcorro_diag256.so > gpurun_out/diag2/impact.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/diag_merge.py tools/_variants/libcorro_diag64.so > gpurun_out/diag2/plain.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/diag2/impact.log | tail -4; grep -v amdgpu.ids gpurun_out/diag2/plain.log | tail -4
