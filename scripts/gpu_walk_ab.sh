#!/bin/bash
# Overflow walk occupancy A/B on config 5 (tools/_variants built with -DOVF_WALK_WAVES=2 / 8; default 4),
# kernel traces of each. Each GPU step has its own limit.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/wab; export TMPDIR=/tmp
for v in default walk2 walk8; do
  lib=""; [ "$v" != default ] && lib="$PWD/tools/_variants/libcorro_$v.so"
  CORRO_HIP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/wab/$v -o run -- python tools/bench_config5.py --sizes 64000000 --reps 3 > gpurun_out/wab/$v.log 2>&1 || { tail -20 gpurun_out/wab/$v.log; exit 1; }
  echo "$v $(grep '^n=' gpurun_out/wab/$v.log | cut -c1-80)"
  python tools/kstats.py gpurun_out/wab/$v | grep ovf_walk
done
