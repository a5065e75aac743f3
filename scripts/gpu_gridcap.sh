#!/bin/bash
# Config 5: workgroups per device-wide overflow pass (CORRO_OVF_GRID_CAP A/B), kernel traces of each.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/gc; export TMPDIR=/tmp
for c in 8192 2048 32768 131072; do
  CORRO_OVF_GRID_CAP=$c timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gc/$c -o run -- python tools/bench_config5.py --sizes 64000000 --reps 3 > gpurun_out/gc/$c.log 2>&1 || { tail -20 gpurun_out/gc/$c.log; exit 1; }
  echo "CAP=$c $(grep '^n=' gpurun_out/gc/$c.log | cut -c1-80)"
  python tools/kstats.py gpurun_out/gc/$c | grep -E "ovf_loadhash|ovf_walk|ovf_gather|ovf_classify|ovf_cgather|ovf_ckeys" | sed 's/  */ /g' | cut -c1-90
done
