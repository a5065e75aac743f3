#!/bin/bash
# Config 5 (adversarial) timing probe + kernel trace. Each GPU step has its own limit.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/c5; export TMPDIR=/tmp
SIZES="${SIZES:-16000000,64000000}"
timeout -k 10 300 python -u tools/bench_config5.py --sizes $SIZES --reps 3 > gpurun_out/c5/probe.log 2>&1 || { tail -20 gpurun_out/c5/probe.log; exit 1; }
cat gpurun_out/c5/probe.log | grep -v amdgpu.ids
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5/trace -o run -- python tools/bench_config5.py --sizes ${TSIZE:-64000000} --reps 2 > gpurun_out/c5/trace.log 2>&1 || { tail -20 gpurun_out/c5/trace.log; exit 1; }
f=$(find gpurun_out/c5/trace -name '*kernel_stats.csv' | head -1); cut -d, -f1-5 "$f" | head -30
