#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u bench_extract.py > gpurun_out/bench_extract.log 2>&1 || exit $?
tail -1 gpurun_out/bench_extract.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/xprof -o run -- python bench_extract.py --steps 3 --warmup 1 > gpurun_out/xprof.log 2>&1 || exit $?
python tools/kstats.py gpurun_out/xprof | head -30
