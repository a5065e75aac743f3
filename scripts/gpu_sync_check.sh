cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_sync.py -x -v --timeout 120 --timeout-method thread > gpurun_out/sync_tests.log 2>&1; rc=$?; tail -5 gpurun_out/sync_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench_sync.py --steps 5 --warmup 2 --one-pass > gpurun_out/bench_sync_1p.log 2>&1 || exit $?
tail -1 gpurun_out/bench_sync_1p.log
timeout -k 10 300 python -u bench_sync.py --steps 5 --warmup 2 > gpurun_out/bench_sync_2p.log 2>&1 || exit $?
tail -1 gpurun_out/bench_sync_2p.log
