#!/bin/bash
# One parameterised GPU-box runner (replaces the per-experiment helpers of rounds 1-3).
#
#   gpurun --timeout 1200 -- 'OUT=r04a bash scripts/gpu.sh smoke tests bench c5imp'
#
# Each named step runs under its own time limit, writes gpurun_out/$OUT/<step>.log and prints the
# last lines; the first failing step ends the script (no GPU step runs after a fault or timeout).
# Steps:
#   smoke      __graft_entry__.smoke()
#   tests      every -m gpu test (TESTS= narrows it, e.g. TESTS="tests/test_gpu_agent_device.py")
#   bench      python bench.py (defaults: config 2, live PMC traffic, cpu baseline)
#   multi2     the N > 1 line rehearsed with 2 gloo ranks on the one GPU (2^26 global changes)
#   quick      python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-pmc
#   trace      kernel trace + stats of a short bench run (gpurun_out/$OUT/trace)
#   pmc        FETCH_SIZE / WRITE_SIZE / SQ groups over a short bench run, one pass each
#   c5 / c5imp config 5 at 64M (no impacts / with impacts), live PMC traffic (SIZES= overrides)
#   c5trace    kernel trace of config 5 (IMPACT=1 for the impact form)
#   agent      tools/bench_agent.py with stage times (agent_path + agent_e2e + mixed)
#   agenttrace kernel trace of tools/bench_agent.py
#   sync       bench_sync.py (config 4) ; synctrace: its kernel trace ; syncpmc: its WRITE/FETCH
#   wire / extract   bench_wire.py / bench_extract.py
#   diag       python $DIAG (any script: one-off measurements under tools/)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT="gpurun_out/${OUT:-run}"
mkdir -p "$OUT"
B="python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-pmc"
C5="python tools/bench_config5.py --sizes ${SIZES:-64000000} --reps 3"
SY="python bench_sync.py --steps 3 --warmup 1 --cpu-sample 1000"

step() {
  local name=$1 secs=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  grep -v amdgpu.ids "$OUT/$name.log" | tail -n "${TAILN:-4}" | cut -c1-2000
  if [ $rc -ne 0 ]; then echo "FAIL $name rc=$rc"; exit $rc; fi
}
kstats() { python tools/kstats.py "$1" 2>/dev/null | head -"${KN:-30}" || true; }

for s in "$@"; do
  case $s in
    smoke) step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) step tests 1100 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread ;;
    bench) step bench 600 python -u bench.py ;;
    multi2) CORRO_BENCH_BACKEND=gloo step multi2 600 python -u bench.py --gpus 2 --changes $((1 << 26)) --steps 3 --warmup 1 ;;
    quick) step quick 300 $B ;;
    trace) step trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- $B
           kstats "$OUT/trace" ;;
    pmc) for g in FETCH_SIZE WRITE_SIZE; do
           step "pmc_$g" 120 rocprofv3 --pmc $g --output-format csv -d "$OUT/pmc_$g" -o run -- $B
         done ;;
    c5) step c5 500 $C5 --pmc ;;
    c5imp) step c5imp 500 $C5 --pmc --impact ;;
    c5trace) step c5trace 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c5trace" -o run -- \
               $C5 ${IMPACT:+--impact}
             kstats "$OUT/c5trace" ;;
    agent) CORRO_AGENT_PROFILE=1 step agent 400 python -u tools/bench_agent.py ;;
    agenttrace) step agenttrace 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/agenttrace" -o run -- \
                  python tools/bench_agent.py
                kstats "$OUT/agenttrace" ;;
    agentsplit) for w in path e2e; do  # separate kernel traces of agent_path and agent_e2e
                  CORRO_AGENT_ONLY=$w step "agent_$w" 400 rocprofv3 --kernel-trace --stats --output-format csv \
                    -d "$OUT/agent_$w" -o run -- python tools/bench_agent.py
                  kstats "$OUT/agent_$w"
                done ;;
    sync) step sync 400 python -u bench_sync.py ;;
    synctrace) step synctrace 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/synctrace" -o run -- $SY
               kstats "$OUT/synctrace" ;;
    syncpmc) for g in FETCH_SIZE WRITE_SIZE; do
               step "syncpmc_$g" 120 rocprofv3 --pmc $g --output-format csv -d "$OUT/syncpmc_$g" -o run -- $SY
             done ;;
    wire) step wire 300 python -u bench_wire.py ;;
    extract) step extract 300 python -u bench_extract.py ;;
    diag) step diag "${DIAG_SECS:-300}" python -u $DIAG ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "=== done"
