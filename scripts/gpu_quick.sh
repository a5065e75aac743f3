#!/bin/bash
# Quick GPU check: GPU parity tests, then the bench (optionally with extra env settings per run).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?; tail -3 gpurun_out/tests.log; [ $rc -ne 0 ] && exit $rc
for v in ${BENCH_VARIANTS:-default}; do
  if [ "$v" = default ]; then env_kv=""; else env_kv="$v"; fi
  echo "=== bench $v"
  env $env_kv timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_$v.log 2>&1 || exit $?
  python - "gpurun_out/bench_$v.log" <<'PY'
import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d=json.loads(l); r=d['roofline']
        print("ms/step %.3f pipeline %.3f frac %.4f" % (d['ms_per_step'], r['pipeline_ms'], r['frac']), {k: round(v,3) for k,v in r['kernels_ms'].items()})
PY
done
if [ -n "$PROF" ]; then
  echo "=== rocprofv3 kernel trace"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/qprof -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/qprof.log 2>&1 || exit $?
  python - <<'PY'
import csv, glob
f = sorted(glob.glob('gpurun_out/qprof/**/run_kernel_stats.csv', recursive=True) + glob.glob('gpurun_out/qprof/run_kernel_stats.csv'))[-1]
for r in csv.DictReader(open(f)):
    if 'corro' in r['Name']: print("%-40s calls %3s avg %9.1f us" % (r['Name'].split('(')[0][-40:], r['Calls'], float(r['AverageNs'])/1e3))
PY
fi
