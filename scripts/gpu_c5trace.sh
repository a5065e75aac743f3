#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/c5; export TMPDIR=/tmp
rm -rf gpurun_out/c5/trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5/trace -o run -- python tools/bench_config5.py --sizes ${TSIZE:-64000000} --reps 2 > gpurun_out/c5/trace.log 2>&1 || { tail -20 gpurun_out/c5/trace.log; exit 1; }
grep "n=" gpurun_out/c5/trace.log
