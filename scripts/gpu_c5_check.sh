#!/bin/bash
# Config 5 timing + kernel trace, then the overflow parity tests and both 64M config-5 folds.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/c5c; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5c/trace -o run -- python tools/bench_config5.py --sizes 64000000 --reps 3 > gpurun_out/c5c/c5.log 2>&1 || { tail -20 gpurun_out/c5c/c5.log; exit 1; }
grep '^n=' gpurun_out/c5c/c5.log | cut -c1-100
python tools/kstats.py gpurun_out/c5c/trace | head -8 | sed 's/  */ /g'
timeout -k 10 400 python -u -m pytest tests/test_gpu_merge.py tests/test_gpu_ovf_reduce.py tests/test_gpu_long.py tests/test_gpu_affinity.py tests/test_gpu_touched.py tests/test_gpu_pk.py tests/test_gpu_dist.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/c5c/tests.log 2>&1
rc=$?; tail -3 gpurun_out/c5c/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest "tests/test_gpu_scale.py::test_config5_64m_two_batch_fold_vs_sharded_oracle" -m gpu -x -q --timeout 280 --timeout-method thread > gpurun_out/c5c/scale.log 2>&1
rc=$?; tail -3 gpurun_out/c5c/scale.log; exit $rc
