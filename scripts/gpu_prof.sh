#!/bin/bash
# rocprofv3 summaries for the config-2 bench: kernel trace + stats, then PMC passes (one per group),
# then the config-4 sync-need bench with its own kernel trace. Each GPU step has its own limit; a
# timeout / abort / crash ends the script.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
B="python bench.py --steps 3 --warmup 1 --no-cpu-baseline"
run() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 $secs "$@" > gpurun_out/prof/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -2 gpurun_out/prof/$name.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
run trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace -o run -- $B
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" "SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM"; do
  tag=$(echo $grp | tr ' ' '_' | cut -c1-40)
  run pmc_$tag 300 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/prof/pmc_$tag -o run -- $B
done
if [ -n "$SYNC" ]; then
  run sync_bench 300 python bench_sync.py
  run sync_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/sync_trace -o run -- python bench_sync.py --steps 3 --warmup 1 --cpu-sample 1000
  run sync_pmc_FETCH 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof/sync_pmc_FETCH -o run -- python bench_sync.py --steps 2 --warmup 1 --cpu-sample 1000
  run sync_pmc_WRITE 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof/sync_pmc_WRITE -o run -- python bench_sync.py --steps 2 --warmup 1 --cpu-sample 1000
fi
if [ -n "$C5" ]; then
  run c5_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/c5_trace -o run -- python tools/bench_config5.py --sizes 16000000
fi
echo "=== done"
