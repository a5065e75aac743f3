#!/bin/bash
# rocprofv3 kernel trace + PMC passes (one group per run) of the config-4 sync bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/sprof
export TMPDIR=/tmp
B="python bench_sync.py --steps 2 --warmup 1 --cpu-sample 1000"
run() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 $secs "$@" > gpurun_out/sprof/$name.log 2>&1; local rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then tail -3 gpurun_out/sprof/$name.log; exit $rc; fi; }
run trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sprof/trace -o run -- $B
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_VALU"; do
  tag=$(echo $grp | tr ' ' '_' | cut -c1-40)
  run pmc_$tag 300 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/sprof/pmc_$tag -o run -- $B
done
echo "=== done"
