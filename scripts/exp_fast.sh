cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/exp
for e in 0 1 2 3 4 8 16 31; do
  echo "== exp $e"
  CORRO_HIP_EXP=$e timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-pmc > gpurun_out/exp/b$e.log 2>&1 || { echo FAIL $e; tail -5 gpurun_out/exp/b$e.log; exit 1; }
  python -c "
import json,sys
for l in open('gpurun_out/exp/b$e.log'):
    if l.startswith('{'):
        d=json.loads(l); r=d['roofline']['kernels_ms']; print('ms/step %.3f'%d['ms_per_step'], {k: round(v,3) for k,v in r.items()}, 'steady', round(d['steady_state']['ms'],3))
"
done
