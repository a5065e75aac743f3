#!/bin/bash
# Need walk with register-held holes: parity (default build, NEED_RH=4), then config 4 per variant.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/rh; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sync.py tests/test_gpu_scale.py -k "sync or config4" -x -q --timeout 300 --timeout-method thread > gpurun_out/rh/tests.log 2>&1 || { tail -20 gpurun_out/rh/tests.log; exit 1; }
tail -2 gpurun_out/rh/tests.log
for v in default ${VARIANTS:-rh0 rh2 rh4w5}; do
  lib=""; [ "$v" != default ] && lib=tools/_variants/libcorro_$v.so
  CORRO_HIP_LIB=$lib timeout -k 10 300 python -u bench_sync.py --cpu-sample 1000 > gpurun_out/rh/b_$v.log 2>&1 || { tail -5 gpurun_out/rh/b_$v.log; exit 1; }
  echo "$v $(grep '^{' gpurun_out/rh/b_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(d["ms_per_step"],3), round(r["kernels_ms"],3), r.get("traffic_by_kernel",{}).get("k_needs_packed"))')"
done
