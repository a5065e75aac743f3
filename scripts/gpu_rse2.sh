#!/bin/bash
# Config 5: OVF_RS_E 16 (new default) vs 32, then the overflow parity tests with the new default.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/rse2; export TMPDIR=/tmp
for v in default rse32; do
  lib=""; [ "$v" != default ] && lib="$PWD/tools/_variants/libcorro_$v.so"
  CORRO_HIP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rse2/$v -o run -- python tools/bench_config5.py --sizes 64000000 --reps 3 > gpurun_out/rse2/$v.log 2>&1 || { tail -20 gpurun_out/rse2/$v.log; exit 1; }
  echo "$v $(grep '^n=' gpurun_out/rse2/$v.log | cut -c1-80)"
  python tools/kstats.py gpurun_out/rse2/$v | grep -E "ovf_lookup"
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_merge.py tests/test_gpu_ovf_reduce.py tests/test_gpu_long.py tests/test_gpu_affinity.py tests/test_gpu_touched.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/rse2/tests.log 2>&1
rc=$?; tail -3 gpurun_out/rse2/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest "tests/test_gpu_scale.py::test_config5_64m_two_batch_fold_vs_sharded_oracle" -m gpu -x -q --timeout 280 --timeout-method thread > gpurun_out/rse2/scale.log 2>&1
rc=$?; tail -3 gpurun_out/rse2/scale.log; exit $rc
