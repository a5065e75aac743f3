#!/bin/bash
# Config-4 write traffic by store kind (diagnostic variants: no kind stores / no range stores / neither).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/sd; export TMPDIR=/tmp
for v in ${VARIANTS:-nd1 nd2 nd3}; do
  CORRO_HIP_LIB=tools/_variants/libcorro_$v.so timeout -k 10 300 python -u bench_sync.py --cpu-sample 1000 > gpurun_out/sd/b_$v.log 2>&1 || { tail -5 gpurun_out/sd/b_$v.log; exit 1; }
  echo "$v $(grep '^{' gpurun_out/sd/b_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(d["ms_per_step"],3), r.get("traffic_by_kernel"))')"
done
