#!/bin/bash
# Config 4 per need-walk variant, twice each, one box.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/rh2; export TMPDIR=/tmp
for pass in 1 2; do
for v in ${VARIANTS:-rh0 rh2 rh3 rh4 rh2w7}; do
  CORRO_HIP_LIB=tools/_variants/libcorro_$v.so timeout -k 10 300 python -u bench_sync.py --cpu-sample 1000 > gpurun_out/rh2/b_${v}_$pass.log 2>&1 || { tail -5 gpurun_out/rh2/b_${v}_$pass.log; exit 1; }
  echo "$pass $v $(grep '^{' gpurun_out/rh2/b_${v}_$pass.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(d["ms_per_step"],3), round(r["kernels_ms"],3), r.get("traffic_by_kernel",{}).get("k_needs_packed"))')"
done
done
