#!/bin/bash
# Config 5: records per thread of the row-summary workgroups (OVF_RS_E 4 / 8 / 16) A/B with kernel traces.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/rse; export TMPDIR=/tmp
for v in default rse4 rse16; do
  lib=""; [ "$v" != default ] && lib="$PWD/tools/_variants/libcorro_$v.so"
  CORRO_HIP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rse/$v -o run -- python tools/bench_config5.py --sizes 64000000 --reps 3 > gpurun_out/rse/$v.log 2>&1 || { tail -20 gpurun_out/rse/$v.log; exit 1; }
  echo "$v $(grep '^n=' gpurun_out/rse/$v.log | cut -c1-80)"
  python tools/kstats.py gpurun_out/rse/$v | grep -E "ovf_lookup|ovf_loadhash"
done
timeout -k 10 400 python -u bench_sync.py > gpurun_out/rse/sync.log 2>&1 || { tail -20 gpurun_out/rse/sync.log; exit 1; }
grep -v amdgpu.ids gpurun_out/rse/sync.log | tail -2 | cut -c1-400
