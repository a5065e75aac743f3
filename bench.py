"""Headline benchmark: merged column-changes/s of the batched crsql_changes merge on MI355X.

N = 1 (default): BASELINE.json configs[1] = config 2 -- 64M (2^26) column changes, 1 table with 4
INTEGER columns, 1000 actors, pk uniform in [1, 2^22], col_version uniform [1, 8], 1/8 of values
from {0..7} (value ties), cl = 1, 64 changes per version per actor.
Synthetic data generated directly in HBM. One step = one `process_multiple_changes`-sized apply of
the whole batch into an empty state (state reset + corro_apply_batch), inputs resident in HBM.

N > 1: `python bench.py --gpus N` launches N fresh ranks itself (one process per GPU; the parent
never touches the GPU) unless it already runs under torchrun (WORLD_SIZE set). Default workload is
config 3, STRONG scaling: 2^29 global changes (pk space 2^25, same distribution), the batch arriving
rank-major (rank r holds the global slice r). One step = pk-hash partition into packed 48-B records
(HIP) + ONE RCCL all-to-all-v of the records over xGMI + unpack + the local merge of the owned rows
-- the exchange is inside the timed region and also reported as `exchange_ms`. The owner-routed
figure (each rank merging only its own rows, no collective on the data path) is reported beside it
as `owner_routed`. `--mode weak` keeps 64M changes per GPU instead.

Roofline: algorithmic bytes (48 B per change + 48 B per output cell) over the apply
pipeline's device time (HIP events on the engine's stream). `traffic` = HBM bytes per apply from
rocprofv3 PMC passes (FETCH_SIZE x 2 per the gfx950 correction, + WRITE_SIZE) that this script runs
on itself, in child processes, before it touches the GPU.

Prints ONE JSON line (rank 0).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

N_CHANGES = 1 << 26
N_GLOBAL_C3 = 1 << 29
N_ACTORS = 1000
N_PK = 1 << 22
N_PK_C3 = 1 << 25
N_COLS = 4
N_C5 = 64_000_000          # BASELINE configs[4] at the size config 2's bench uses
C5_PMC_APPLIES = 3
ALG_BYTES_PER_CHANGE = 48  # pk 8, table_cid 4, col_version 8, db_version 8, cl 4, seq 4, site 4, value 8
ALG_BYTES_PER_CELL = 48
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: 8 TB/s spec
METRIC = "merged column-changes/sec (node) at 1/2/4/8 GPUs + % of HBM BW roofline"
# The reference's own CPU apply (cr-sqlite 0.17 through SQLite, one writer, per-change INSERT +
# crsql_rows_impacted()), recorded during the survey in the build container -- not re-run here: the
# cr-sqlite binary ships prebuilt inside the reference and is never loaded.
REFERENCE_CPU = {"value_range": [53000.0, 103000.0], "unit": "merged column-changes/s", "cores": 1,
                 "kind": "reference (survey-recorded)",
                 "sample": "cr-sqlite 0.17.0 via SQLite 3.37.2, 100k-1M changes, 1 table x 3 INTEGER cols: 103k/s "
                           "(100k changes, 4 actors), 53-56k/s (1M changes: B-tree growth); recorded in the build "
                           "container (Intel Xeon, 1 core), SURVEY.md App. D -- not re-run on the GPU box"}


def cpu_baseline(batch_dev, seconds_target=15.0):
    """CPU apply of the same workload on the host cores (SURVEY §8(d) CPU baseline (ii)):
    the oracle's cr-sqlite fold restatement (kind 'port'), pk-sharded over the host threads on the
    bench's own 2^26-change batch (value, `cores` = threads used), plus the sequential 1-core fold —
    the reference's single-writer shape (agent.rs:480-482) — on a bounded sample of the same
    distribution: the largest of 1M..16M changes whose run stays near the target."""
    from oracle import oracle as O
    import numpy as np
    import synth
    sites = synth.site_ids(N_ACTORS, 1)
    threads = max(1, min(os.cpu_count() or 1, int(os.environ.get("OMP_NUM_THREADS") or 16)))
    hb = {k: v.cpu().numpy() for k, v in batch_dev.items()}
    for k in ("table_cid", "cl", "seq", "site"):
        hb[k] = hb[k].view(np.uint32)
    for k in ("pk", "val0"):
        hb[k] = hb[k].view(np.uint64)
    n_all = len(hb["pk"])
    g = O.ShardedFold(sites, nshards=4 * threads, nthreads=threads)
    t0 = time.perf_counter()
    g.apply(hb, impact=False)
    dt_mt = time.perf_counter() - t0
    del g, hb
    best = None
    n = 1 << 20
    while True:
        b = synth.uniform_batch(n, N_ACTORS, N_PK, N_COLS, 7 + n)
        f = O.Fold(sites)
        t0 = time.perf_counter()
        f.apply(b)
        dt = time.perf_counter() - t0
        best = (n, dt)
        del f, b
        if dt * 2 > seconds_target or n >= (1 << 24):
            break
        n *= 2
    n, dt = best
    return {"value": n_all / dt_mt, "unit": "merged column-changes/s", "cores": threads, "kind": "port",
            "sample": f"the bench's own {n_all}-change batch folded by oracle/crsql_fold.c of_apply_sharded "
                      f"({4 * threads} pk-hash shards, {threads} threads) in {dt_mt:.2f} s",
            "single_core": {"value": n / dt, "cores": 1,
                            "sample": f"{n} changes of the config-2 distribution folded sequentially in {dt:.2f} s"},
            "reference": REFERENCE_CPU}


def cpu_baseline_sample(npk, n=1 << 24, threads=None):
    """The N > 1 lines' CPU baseline, bounded to a few seconds: the oracle's fold restatement (kind
    'port') pk-sharded over the host threads on a 16M-change sample of the line's distribution."""
    from oracle import oracle as O
    import synth
    sites = synth.site_ids(N_ACTORS, 1)
    threads = threads or max(1, min(os.cpu_count() or 1, int(os.environ.get("OMP_NUM_THREADS") or 16)))
    b = synth.uniform_batch(n, N_ACTORS, npk, N_COLS, 11 + n)
    g = O.ShardedFold(sites, nshards=4 * threads, nthreads=threads)
    t0 = time.perf_counter()
    g.apply(b, impact=False)
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "merged column-changes/s", "cores": threads, "kind": "port",
            "sample": f"{n} changes of the line's distribution (pk space {npk}) folded by oracle/crsql_fold.c "
                      f"of_apply_sharded ({4 * threads} pk-hash shards, {threads} threads) in {dt:.2f} s",
            "reference": REFERENCE_CPU}


# ------------------------------------------------------------------------------------- PMC traffic
def _ours(kernel_name):
    """Kernels of the apply pipeline (the library's own and the rocPRIM sorts it launches), not the
    synthetic-data generation or torch's memsets."""
    return kernel_name.startswith("k_") or "corro" in kernel_name or "rocprim" in kernel_name


def _short_kernel(name):
    name = name.replace("(anonymous namespace)::", "").split("(")[0]
    name = name.replace("void ", "").replace("corro::", "")
    return "rocprim" if "rocprim" in name else name


def _read_counter(dirname, counter):
    """(total, {kernel: total}) of one counter over the pipeline's kernels, or None."""
    import csv
    import glob
    files = glob.glob(os.path.join(dirname, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        return None
    tot, per = 0.0, {}
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") == counter and _ours(r.get("Kernel_Name", "")):
                v = float(r["Counter_Value"])
                tot += v
                k = _short_kernel(r["Kernel_Name"])
                per[k] = per.get(k, 0.0) + v
    return tot, per


def pmc_traffic_live(changes, applies=3, timeout=240, child_cmd=None):
    """HBM bytes per apply measured now: two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE: they do
    not fit one pass) over a child run of this bench doing `applies` applies of the same workload.
    Counters are KiB; FETCH_SIZE is doubled (gfx950 reports half of wide coalesced reads,
    MI355X_MICROARCH.md §HBM). Runs BEFORE this process touches the GPU. Returns (bytes or None,
    note)."""
    import shutil
    import tempfile
    rp = shutil.which("rocprofv3") or ("/opt/rocm/bin/rocprofv3" if os.path.exists("/opt/rocm/bin/rocprofv3") else None)
    if not rp:
        return None, "rocprofv3 not found", None
    tmp = os.environ.get("TMPDIR") or "/tmp"
    got, per = {}, {}
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        d = tempfile.mkdtemp(prefix="corro_pmc_", dir=tmp)
        child = child_cmd or [os.path.abspath(__file__), "--pmc-child", "--changes", str(changes), "--steps",
                              str(applies - 1), "--warmup", "1"]
        cmd = ["timeout", "-k", "10", "-s", "KILL", str(timeout), rp, "--pmc", counter, "--output-format", "csv",
               "-d", d, "-o", "run", "--", sys.executable] + child
        try:
            r = subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, timeout=timeout + 30)
        except subprocess.TimeoutExpired:
            return None, f"rocprofv3 --pmc {counter} timed out", None
        v = _read_counter(d, counter)
        shutil.rmtree(d, ignore_errors=True)
        if r.returncode != 0 or v is None:
            return None, f"rocprofv3 --pmc {counter} rc={r.returncode}: {r.stderr.decode(errors='replace')[-300:]}", None
        got[counter] = v[0] / applies
        scale = (2.0 if counter == "FETCH_SIZE" else 1.0) * 1024.0 / applies
        for k, x in v[1].items():
            per.setdefault(k, {"fetch": 0.0, "write": 0.0})["fetch" if counter == "FETCH_SIZE" else "write"] = x * scale
    return (2 * got["FETCH_SIZE"] + got["WRITE_SIZE"]) * 1024.0, \
        f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes run by bench.py on itself ({applies} applies each)", per


# ----------------------------------------------------------------------------------- self-launch
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(n, script=None):
    """One fresh process per GPU (this parent never initialises the GPU): RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_* as torchrun sets them. Returns the worst exit code."""
    port = str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(script or __file__)] + sys.argv[1:], env=env))
    rcs = [p.wait() for p in procs]
    return max(rcs, key=abs)


# ------------------------------------------------------------------------------------------ main
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--changes", type=int, default=None,
                    help="N=1: changes per apply (default 2^26); N>1 strong: global changes (default 2^29)")
    ap.add_argument("--mode", choices=("strong", "weak"), default="strong",
                    help="N>1: strong = config 3 (2^29 global, exchange timed); weak = 64M per GPU, owner-routed")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pmc", action="store_true", help="skip the live rocprofv3 traffic passes")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--pmc-rank-child", type=int, default=0, help=argparse.SUPPRESS)  # world size emulated
    ap.add_argument("--pmc-c5-child", type=int, default=-1, help=argparse.SUPPRESS)  # 0 / 1: config 5 (impacts)
    ap.add_argument("--no-config5", action="store_true", help="skip the config-5 figure of the N = 1 line")
    args = ap.parse_args()
    if args.pmc_rank_child:
        run_rank_child(args, args.pmc_rank_child)
        return
    if args.pmc_c5_child >= 0:
        config5(bool(args.pmc_c5_child), reps=args.steps, child=True)
        return

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus and not args.pmc_child:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; measuring {world} rank(s)", file=sys.stderr)
    rank = int(os.environ.get("RANK", "0"))

    traffic, traffic_note, traffic_kern = None, "not measured (--no-pmc)", None
    c5_traffic = {}
    if world == 1 and not args.pmc_child and not args.no_pmc and rank == 0:
        traffic, traffic_note, traffic_kern = pmc_traffic_live(args.changes or N_CHANGES)
        if not args.no_config5:
            for imp in (0, 1):
                child = [os.path.abspath(__file__), "--pmc-c5-child", str(imp), "--steps", str(C5_PMC_APPLIES - 1)]
                c5_traffic[imp] = pmc_traffic_live(N_C5, applies=C5_PMC_APPLIES, timeout=300, child_cmd=child)

    if world > 1 and not args.no_pmc and rank == 0:
        # per-rank traffic of the step's local kernels, before this rank touches its GPU (the other
        # ranks wait in the process-group rendezvous meanwhile)
        G = (args.changes or N_GLOBAL_C3) if args.mode == "strong" else (args.changes or N_CHANGES) * world
        child = [os.path.abspath(__file__), "--pmc-rank-child", str(world), "--changes", str(G), "--mode", args.mode,
                 "--steps", "2", "--warmup", "1"]
        traffic, traffic_note, traffic_kern = pmc_traffic_live(G // world, applies=3, child_cmd=child)

    if world == 1:
        run_single(args, traffic, traffic_note, traffic_kern, c5_traffic)
    else:
        run_multi(args, world, rank, (traffic, traffic_note, traffic_kern))


def rank_capacity(n_local, G, npk, world):
    """A rank engine's capacity hint: its batch, or enough for the rows it will own (npk pks drawn G
    times, 1/world of them owned; the row store sizes its regions for hint / 16 rows), so the store
    does not grow (k_rehash) inside the timed step."""
    import math
    rows = npk * (1.0 - math.exp(-G / max(1, npk))) / world
    return int(max(n_local, 16 * rows * 1.1, 1))


def run_rank_child(args, world):
    """(PMC child) one rank's local kernels of the N > 1 step on one GPU: rank 0's slice, the slot
    partition for `world` destinations, the unpack of an equal-size received slot buffer (its own
    slots stand in for the peers': the same bytes and counts) and the mapped merge. The all-to-alls
    are not run: RCCL's copies are not the library's kernels."""
    import torch
    import synth
    import corrosion_amd as ca
    from corrosion_amd.dist import slot_cap
    strong = args.mode == "strong"
    G = args.changes
    n_local = G // world
    npk = N_PK_C3 if strong else N_PK * world
    # (its own slots stand in for the received ones, so it merges every row of its slice -- more distinct
    # rows than the rank owns: the engine is presized for those, as a real rank's is for its own)
    eng = ca.MergeEngine({"t": ["a", "b", "c", "d"]}, capacity_hint=rank_capacity(n_local, n_local, npk, 1), device=0)
    eng.register_sites(synth.site_ids(N_ACTORS, 1))
    batch = synth.uniform_batch_torch(n_local, N_ACTORS, npk, N_COLS, seed=synth.config_seed(3), device="cuda:0",
                                      offset=0, global_n=G)
    cap = slot_cap(n_local, world)
    for _ in range(args.warmup + args.steps):
        eng.reset()
        recs, cnt = eng.partition_slots(batch, world, cap)
        eng.apply_slots(recs, world, cap, cnt)
    torch.cuda.synchronize()
    eng.close()


def config5(impact, reps=3, child=False, traffic=None):
    """BASELINE configs[4] (adversarial mix) on one GPU: 64M changes generated in HBM
    (synth.adversarial_batch_torch: 8 tables of (INTEGER, INTEGER, BLOB, BLOB) columns, Zipf(1.1) pks
    over 2^20, 30 % sentinel deletes / resurrects, mixed value classes), one apply into an empty state
    per rep, with or without impact flags. Returns (median ms, cells, stage ms). child: the PMC child
    (warm-up + `reps` applies, nothing printed)."""
    import torch
    import synth
    import corrosion_amd as ca
    seed = synth.config_seed(5)
    batch = synth.adversarial_batch_torch(N_C5, N_ACTORS, 8, 1 << 20, seed, device="cuda:0")
    eng = ca.MergeEngine(synth.adversarial_schema(8), capacity_hint=N_C5, device=0)
    eng.register_sites(synth.site_ids(N_ACTORS, seed))
    eng.set_profiling(True)
    prep = eng.prepare(batch, impact=impact)
    times, stages = [], []
    for rep in range(reps + 1):
        eng.reset()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.apply_prepared(prep)
        torch.cuda.synchronize()
        if rep:
            times.append((time.perf_counter() - t0) * 1e3)
            stages.append(eng.last_timings())
    cells = eng.count()
    eng.close()
    if child:
        return None
    k = sorted(range(len(times)), key=times.__getitem__)[len(times) // 2]
    return times[k], cells, stages[k]


def config5_figures(reps, c5_traffic):
    """The config-5 object of the N = 1 line: ms per apply without and with impact flags, traffic
    ratio (live PMC bytes per apply over SURVEY §8(d)'s 56 B per change and per output cell)."""
    out = {"workload": "config 5: 64M changes, 8 tables, Zipf(1.1) pks over 2^20, 30 percent sentinels, mixed "
                       f"values; one apply into an empty state (median of {reps})", "changes": N_C5}
    for imp in (0, 1):
        ms, cells, st = config5(bool(imp), reps=reps)
        alg = 56 * (N_C5 + cells)
        tr = c5_traffic.get(imp, (None, "not measured", None))
        key = "impact" if imp else "no_impact"
        out[key] = {"ms": ms, "changes_per_s": N_C5 / (ms * 1e-3), "cells": int(cells), "alg_bytes": alg,
                    "roofline_frac": alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, "stages_ms": st,
                    "traffic": tr[0], "traffic_ratio": (tr[0] / alg) if tr[0] else None, "traffic_source": tr[1],
                    "traffic_by_kernel": ({k: {"fetch": round(v["fetch"]), "write": round(v["write"])}
                                           for k, v in sorted(tr[2].items())} if tr[2] else None)}
    out["ms"] = out["no_impact"]["ms"]
    out["ms_impact"] = out["impact"]["ms"]
    out["traffic_ratio"] = out["no_impact"]["traffic_ratio"]
    out["traffic_ratio_impact"] = out["impact"]["traffic_ratio"]
    return out


def blob_pk_figures(int_ms, reps=5):
    """Config 2 over a testsblob-shaped table (corro-tests/src/lib.rs:32-35): the same 2^26 changes with
    every pk a 16-byte BLOB packed in HBM (19 bytes, synth.blob_pks_torch), interned on the device
    (corro_pk_keys_device) and applied. `cold`: the first intern of the batch's 4.2 M keys into an
    empty table; `intern_ms`: a warm intern (every key already held, a node's steady state); `apply_ms`:
    reset + apply with the interned keys; `e2e_ms`: warm intern + reset + apply, against the INTEGER-pk
    step (`int_ms`)."""
    import torch
    import synth
    import corrosion_amd as ca
    n = N_CHANGES
    b = synth.uniform_batch_torch(n, N_ACTORS, N_PK, N_COLS, seed=synth.config_seed(2), device="cuda:0")
    data, off = synth.blob_pks_torch(b["pk"])
    eng = ca.MergeEngine({"t": ["a", "b", "c", "d"]}, capacity_hint=n, device=0, interned=("t",))
    eng.register_sites(synth.site_ids(N_ACTORS, 1))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    keys = eng.pk_keys_device("t", data, off)
    torch.cuda.synchronize()
    cold = (time.perf_counter() - t0) * 1e3
    b["pk"] = keys
    prep = eng.prepare(b)
    it, ap, ee = [], [], []
    for _ in range(reps + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.pk_keys_device("t", data, off)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        eng.reset()
        eng.apply_prepared(prep)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        it.append((t1 - t0) * 1e3)
        ap.append((t2 - t1) * 1e3)
        ee.append((t2 - t0) * 1e3)
    med = lambda x: sorted(x[1:])[len(x[1:]) // 2]
    out = {"workload": "config 2 with 16-byte BLOB pks (testsblob shape), packed in HBM", "changes": n,
           "keys": int(keys.max().item()) + 1, "intern_cold_ms": cold, "intern_ms": med(it), "apply_ms": med(ap),
           "e2e_ms": med(ee), "int_pk_ms": int_ms, "apply_ratio": med(ap) / int_ms, "e2e_ratio": med(ee) / int_ms}
    eng.close()
    return out


def run_single(args, traffic, traffic_note, traffic_kern=None, c5_traffic=None):
    import torch
    import synth
    import corrosion_amd as ca
    n = args.changes or N_CHANGES
    dev = torch.device("cuda", 0)
    eng = ca.MergeEngine({"t": ["a", "b", "c", "d"]}, capacity_hint=n, device=0)
    eng.register_sites(synth.site_ids(N_ACTORS, 1))
    batch = synth.uniform_batch_torch(n, N_ACTORS, N_PK, N_COLS, seed=synth.config_seed(2), device=dev)
    torch.cuda.synchronize()
    eng.set_profiling(True)
    # the batch's C-ABI descriptor (device pointers and sizes) is built once: a Rust caller hands
    # the same struct over; every step still resets the state and runs the whole apply
    prep = eng.prepare(batch)

    def step():
        eng.reset()
        eng.apply_prepared(prep)

    for _ in range(args.warmup):
        step()
    if args.pmc_child:
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        eng.close()
        return
    cells = eng.count()
    kern = {}
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        for k, v in eng.last_timings().items():
            kern[k] = kern.get(k, 0.0) + v
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    kern = {k: v / args.steps for k, v in kern.items()}
    pipe_ms = sum(kern.values())
    alg_bytes = ALG_BYTES_PER_CHANGE * n + ALG_BYTES_PER_CELL * cells
    step_ms = dt / args.steps * 1e3
    # (the fraction is over the whole step, reset included; the pipeline-only figure beside it)
    achieved = alg_bytes / (step_ms * 1e-3) / 1e9
    achieved_pipe = alg_bytes / (pipe_ms * 1e-3) / 1e9
    steady = steady_state(eng, prep, n, dev, dt / args.steps * 1e3, cells)
    agent = agent_path(eng, batch, n)
    e2e_agent = agent_e2e(eng, batch, n, agent["ms"])
    mixed_agent = agent_e2e_mixed(eng, batch, n, e2e_agent["ms"], reps=5)
    e2e = host_batch_e2e(eng, batch, n)
    cpu = None if args.no_cpu_baseline else cpu_baseline(batch)
    eng.close()
    del batch, prep
    torch.cuda.empty_cache()
    blob = blob_pk_figures(dt / args.steps * 1e3)
    torch.cuda.empty_cache()
    c5 = None if args.no_config5 else config5_figures(3, c5_traffic or {})
    line = {
        "metric": METRIC,
        "value": n / dt * args.steps,
        "unit": "merged column-changes/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "none",
        "vs_baseline": None,
        "dtype": "int64",
        "data": "synthetic (seeded, generated in HBM)",
        "config": {"workload": "config 2: 64M column-changes, 1 table x 4 INTEGER cols, 1000 actors, uniform pk in "
                               "[1,2^22], cl=1, one apply into an empty state per step",
                   "changes": n, "cells": int(cells), "parallelism": "1 GPU"},
        "roofline": {"bound": "hbm", "kernel": "apply pipeline: " + "+".join(k for k in kern if kern[k] > 0),
                     "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                     "traffic": traffic, "traffic_source": traffic_note,
                     "traffic_ratio": (traffic / alg_bytes) if traffic else None,
                     "traffic_by_kernel": ({k: {"fetch": round(v["fetch"]), "write": round(v["write"])}
                                            for k, v in sorted(traffic_kern.items())} if traffic_kern else None),
                     "achieved_basis": "algorithmic bytes / ms_per_step (reset + apply)",
                     "pipeline_achieved": achieved_pipe, "pipeline_frac": achieved_pipe / HBM_PEAK_GBS,
                     "alg_bytes_per_apply": alg_bytes, "pipeline_ms": pipe_ms, "kernels_ms": kern,
                     "dominant": max(kern, key=kern.get)},
        "cpu_baseline": cpu,
        "steady_state": steady,
        "agent_path": agent,
        "agent_e2e": e2e_agent,
        "agent_e2e_mixed": mixed_agent,
        "end_to_end_h2d": e2e,
        "blob_pk": blob,
        "config5": c5,
    }
    print(json.dumps(line), flush=True)


def host_batch_e2e(eng, batch, n, reps=3):
    """SURVEY §8(d)'s end-to-end figure: the same batch handed over in host memory (numpy arrays, as
    a Rust caller's Vec<Change> columns), so the apply includes the H2D copies of every field.
    Never `value` (the contract measures device-resident inputs)."""
    import torch
    host = {k: v.cpu().numpy() for k, v in batch.items()}
    prep = eng.prepare(host)
    ms = []
    for _ in range(reps):
        eng.reset()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.apply_prepared(prep)
        torch.cuda.synchronize()
        ms.append((time.perf_counter() - t0) * 1e3)
    ms.sort()
    med = ms[len(ms) // 2]
    del host, prep
    return {"ms": med, "changes_per_s": n / (med * 1e-3),
            "note": "config-2 batch from pageable host memory (H2D of every SoA field inside the apply call), "
                    f"empty state, median of {reps}"}


def steady_state(eng, prep, n, dev, empty_ms, cells, reps=3):
    """The same-size config-2 batch (another seed) applied into the populated state the headline
    batch leaves (16.5M cells): the in-place row store's apply cost against the empty-state one."""
    import torch
    import synth
    other = synth.uniform_batch_torch(n, N_ACTORS, N_PK, N_COLS, seed=synth.config_seed(2) + 1, device=dev)
    prep2 = eng.prepare(other)
    ms = []
    for _ in range(reps):
        eng.reset()
        eng.apply_prepared(prep)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.apply_prepared(prep2)
        torch.cuda.synchronize()
        ms.append((time.perf_counter() - t0) * 1e3)
    ms.sort()
    med = ms[len(ms) // 2]
    del other, prep2
    return {"ms": med, "state_cells_before": int(cells), "ratio_vs_empty_state": med / empty_ms,
            "note": "a second 64M config-2 batch applied into the ~16.5M-cell state of the first (median of "
                    f"{reps}); empty-state step = reset + apply"}


def agent_path(eng, batch, n, reps=3):
    """The same batch applied with per-change impact flags (crsql_rows_impacted growth: what
    process_multiple_changes asks for, util.rs:1246-1262) into an empty state; median of `reps`."""
    import torch
    prep = eng.prepare(batch, impact=True)
    ms = []
    for _ in range(reps):
        eng.reset()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.apply_prepared(prep)
        torch.cuda.synchronize()
        ms.append((time.perf_counter() - t0) * 1e3)
    ms.sort()
    med = ms[len(ms) // 2]
    stages = eng.last_timings()
    del prep
    return {"ms": med, "changes_per_s": n / (med * 1e-3), "merge_ms": stages.get("k_merge"),
            "note": f"config-2 batch with impact flags (the agent path), reset + apply, median of {reps}"}


def agent_e2e(eng, batch, n, agent_ms=None, reps=3):
    """The drop-in entry point end to end: config 2 as ChangeV1-shaped input -- 1000 actors x ~1049
    versions x 64 changes, changesets arriving interleaved across actors (round-robin by version) and
    the change batch laid out in that arrival order (as a decoder emits it), every change carrying its
    changeset's NTP64 ts -- through corro_process_multiple_changes with the
    batch left in HBM (CORRO_MEM_DEVICE): header dedup passes and gap bookkeeping on the host (actors in
    parallel), the unknown-name screen, the regroup into ActorId order (gather kernel), the merge with
    impact flags, and the impactful flags / Current-Cleared outcomes on the device. Each rep resets the
    state and starts a fresh Bookie (util.rs:691-1037 on an empty node); median of `reps`."""
    import ctypes as C
    import numpy as np
    import torch
    import synth
    import corrosion_amd as ca
    from corrosion_amd import _lib as L
    per_actor = -(-n // N_ACTORS)
    ids = np.ascontiguousarray(synth.site_ids(N_ACTORS, 1), dtype=np.uint8)   # ordinal a = actor a
    cs_dt = np.dtype([("actor_id", "<u8"), ("site", "<u4"), ("kind", "<u4"), ("version_start", "<u8"),
                      ("version_end", "<u8"), ("seq_start", "<u8"), ("seq_end", "<u8"), ("last_seq", "<u8"),
                      ("ts", "<u8"), ("change_off", "<u8"), ("change_count", "<u8")])
    assert cs_dt.itemsize == C.sizeof(L.Changeset)
    a_idx, v_idx = [], []
    for a in range(N_ACTORS):
        lo, hi = a * per_actor, min(n, (a + 1) * per_actor)
        nv = max(0, -(-(hi - lo) // 64))
        a_idx.append(np.full(nv, a, np.int64))
        v_idx.append(np.arange(nv, dtype=np.int64))
    a_idx, v_idx = np.concatenate(a_idx), np.concatenate(v_idx)
    order = np.lexsort((a_idx, v_idx))                 # arrival: version-major, actors interleaved
    a_idx, v_idx = a_idx[order], v_idx[order]
    off = a_idx * per_actor + v_idx * 64
    cnt = np.minimum(64, np.minimum(n, (a_idx + 1) * per_actor) - off)
    # the batch laid out in arrival order (as a decoder emits it): changeset j at arr[j]
    arr = np.cumsum(cnt) - cnt
    dev = batch["pk"].device
    idx = (torch.repeat_interleave(torch.from_numpy(off - arr).to(dev), torch.from_numpy(cnt).to(dev))
           + torch.arange(n, device=dev))
    cs = np.zeros(len(off), cs_dt)
    cs["actor_id"] = ids.ctypes.data + 16 * a_idx
    cs["site"] = a_idx
    cs["kind"] = L.CORRO_CS_FULL
    cs["version_start"] = cs["version_end"] = v_idx + 1
    cs["seq_end"] = cs["last_seq"] = cnt - 1
    cs["ts"] = ((v_idx + 1) << 32) | a_idx             # NTP64-shaped, per changeset
    cs["change_off"], cs["change_count"] = arr, cnt
    full = {k: v[idx].contiguous() for k, v in batch.items()}
    full["ts"] = ((full["db_version"] << 32) | full["site"].to(torch.int64)).contiguous()
    del idx
    s = L.Changes()
    s.n = n
    for k in ("pk", "table_cid", "col_version", "db_version", "cl", "seq", "site", "val0", "ts"):
        setattr(s, k, full[k].data_ptr())
    imp = torch.zeros(n, dtype=torch.uint8, device=batch["pk"].device)
    # the headers as a decoder leaves them on the device (CORRO_MEM_DEVICE_HEADERS: uploaded once,
    # outside the timed region, like the change batch); known on the device too
    dcs = torch.from_numpy(cs.view(np.uint8).copy()).to(dev)
    dknown = torch.zeros(len(cs), dtype=torch.int32, device=dev)

    def timed(mem):
        known = np.zeros(len(cs), np.int32)
        out = L.ProcessOut()
        out.impactful = imp.data_ptr()
        if mem == L.CORRO_MEM_DEVICE_HEADERS:
            out.known, cs_arg = dknown.data_ptr(), C.c_void_p(dcs.data_ptr())
        else:
            out.known, cs_arg = known.ctypes.data, cs.ctypes.data
        torch.cuda.synchronize()
        ms = []
        for _ in range(reps):
            bk = ca.agent.Bookie()
            eng.reset()
            dknown.fill_(-1)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            L.check(L.lib().corro_process_multiple_changes(eng._h, bk._h, cs_arg, len(cs), C.byref(s), mem,
                                                           C.byref(out)))
            torch.cuda.synchronize()
            ms.append((time.perf_counter() - t0) * 1e3)
            del bk
        first = ms[0]
        ms.sort()
        if mem == L.CORRO_MEM_DEVICE_HEADERS:
            known = dknown.cpu().numpy()
        ok = bool((known == 1).all())      # every version Current (empty state: each one impactful)
        return ms[len(ms) // 2], ok, first

    # (the process's first agent calls: the pinned areas and pools grow in the first call of each mode)
    med_h, ok_h, first_h = timed(L.CORRO_MEM_DEVICE)
    nimp_h = int(imp.sum().item())
    med, ok, first = timed(L.CORRO_MEM_DEVICE_HEADERS)
    nimp = int(imp.sum().item())
    del full, imp, dcs, dknown
    return {"ms": med, "changes_per_s": n / (med * 1e-3), "changesets": int(len(cs)),
            "ratio_vs_agent_path": (med / agent_ms) if agent_ms else None, "all_current": ok,
            "impactful_changes": nimp, "first_call_ms": first,
            "host_headers": {"ms": med_h, "all_current": ok_h, "impactful_changes": nimp_h, "first_call_ms": first_h,
                             "note": "the same call with the headers and known in host memory (CORRO_MEM_DEVICE: a "
                                     "call this large copies the headers in parallel host threads into pinned "
                                     "memory, uploads them chunk by chunk and runs the device header passes)"},
            "note": "corro_process_multiple_changes (CORRO_MEM_DEVICE_HEADERS: changes, headers, known, impactful "
                    "in HBM) on config 2 as 1000 actors x ~1049 versions x 64 changes arriving interleaved (batch "
                    "in arrival order), reset + fresh Bookie + call, median of "
                    f"{reps}; first_call_ms: the first call of the mode (host_headers' is the process's first agent "
                    "call: its pinned areas and the bookie's pool are allocated inside it)"}


def agent_e2e_mixed(eng, batch, n, fast_ms=None, reps=3, resend=0.10, partial=0.05, empty=0.05, seed=5):
    """agent_e2e's call with the slow cases the reference routes through its per-actor checks
    (util.rs:704-884): ~10 % of the versions re-sent later in the same call (pass 1's seen set skips
    them), ~5 % arriving as two partial halves (incomplete: buffered, process_incomplete_version
    util.rs:1053-1186), ~5 % as Empty versions (cleared, crsql_set_db_version when past the max).
    Same changes in HBM, headers in HBM (CORRO_MEM_DEVICE_HEADERS), fresh Bookie and empty state per
    rep; median of `reps`. Reported beside the all-fast figure (ratio_vs_fast)."""
    import ctypes as C
    import numpy as np
    import torch
    import synth
    import corrosion_amd as ca
    from corrosion_amd import _lib as L
    rng = np.random.default_rng(seed)
    per_actor = -(-n // N_ACTORS)
    ids = np.ascontiguousarray(synth.site_ids(N_ACTORS, 1), dtype=np.uint8)
    cs_dt = np.dtype([("actor_id", "<u8"), ("site", "<u4"), ("kind", "<u4"), ("version_start", "<u8"),
                      ("version_end", "<u8"), ("seq_start", "<u8"), ("seq_end", "<u8"), ("last_seq", "<u8"),
                      ("ts", "<u8"), ("change_off", "<u8"), ("change_count", "<u8")])
    a_idx, v_idx = [], []
    for a in range(N_ACTORS):
        lo, hi = a * per_actor, min(n, (a + 1) * per_actor)
        nv = max(0, -(-(hi - lo) // 64))
        a_idx.append(np.full(nv, a, np.int64))
        v_idx.append(np.arange(nv, dtype=np.int64))
    a_idx, v_idx = np.concatenate(a_idx), np.concatenate(v_idx)
    order = np.lexsort((a_idx, v_idx))
    a_idx, v_idx = a_idx[order], v_idx[order]
    off = a_idx * per_actor + v_idx * 64
    cnt = np.minimum(64, np.minimum(n, (a_idx + 1) * per_actor) - off)
    arr = np.cumsum(cnt) - cnt
    dev = batch["pk"].device
    idx = (torch.repeat_interleave(torch.from_numpy(off - arr).to(dev), torch.from_numpy(cnt).to(dev))
           + torch.arange(n, device=dev))
    base = np.zeros(len(off), cs_dt)
    base["actor_id"] = ids.ctypes.data + 16 * a_idx
    base["site"] = a_idx
    base["kind"] = L.CORRO_CS_FULL
    base["version_start"] = base["version_end"] = v_idx + 1
    base["seq_end"] = base["last_seq"] = cnt - 1
    base["ts"] = ((v_idx + 1) << 32) | a_idx
    base["change_off"], base["change_count"] = arr, cnt
    u = rng.random(len(base))
    emp = u < empty
    par = (u >= empty) & (u < empty + partial) & (cnt >= 2)
    cs = base.copy()
    cs["kind"][emp] = L.CORRO_CS_EMPTY
    cs["change_count"][emp] = 0
    h = cnt // 2
    first = cs.copy()[par]
    first["seq_end"] = h[par] - 1
    first["change_count"] = h[par]
    second = base[par].copy()
    second["seq_start"] = h[par]
    second["change_off"] = arr[par] + h[par]
    second["change_count"] = cnt[par] - h[par]
    cs[par] = first
    resent = base[rng.random(len(base)) < resend]
    tail = np.concatenate([second, resent])
    tail = tail[rng.permutation(len(tail))]
    # second halves and re-sends arrive later in the call: spread over the back half of the arrival order
    pos = np.sort(rng.integers(len(cs) // 2, len(cs) + 1, size=len(tail)))
    cs = np.insert(cs, pos, tail)
    full = {k: v[idx].contiguous() for k, v in batch.items()}
    full["ts"] = ((full["db_version"] << 32) | full["site"].to(torch.int64)).contiguous()
    del idx
    s = L.Changes()
    s.n = n
    for k in ("pk", "table_cid", "col_version", "db_version", "cl", "seq", "site", "val0", "ts"):
        setattr(s, k, full[k].data_ptr())
    imp = torch.zeros(n, dtype=torch.uint8, device=dev)
    dcs = torch.from_numpy(cs.view(np.uint8).copy()).to(dev)
    dknown = torch.zeros(len(cs), dtype=torch.int32, device=dev)
    out_ = L.ProcessOut()
    out_.impactful = imp.data_ptr()
    out_.known = dknown.data_ptr()
    ms = []
    nready = 0
    for r in range(reps + 1):  # (the first call untimed: the pool and pinned areas grow there once)
        bk = ca.agent.Bookie()
        eng.reset()
        dknown.fill_(-1)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        L.check(L.lib().corro_process_multiple_changes(eng._h, bk._h, C.c_void_p(dcs.data_ptr()), len(cs), C.byref(s),
                                                       L.CORRO_MEM_DEVICE_HEADERS, C.byref(out_)))
        torch.cuda.synchronize()
        if r:
            ms.append((time.perf_counter() - t0) * 1e3)
        else:
            first = (time.perf_counter() - t0) * 1e3
        nready = int(out_.n_ready)
        del bk
    ms.sort()
    med = ms[len(ms) // 2]
    known = dknown.cpu().numpy()
    kinds = {name: int((known == v).sum()) for name, v in (("current", 1), ("cleared", 2), ("partial", 3),
                                                         ("skipped", 0))}
    del full, imp, dcs, dknown
    return {"ms": med, "changes_per_s": n / (med * 1e-3), "changesets": int(len(cs)),
            "ratio_vs_fast": (med / fast_ms) if fast_ms else None, "first_call_ms": first, "known": kinds,
            "n_ready": nready,
            "mix": {"resent": float(resend), "partial": float(partial), "empty": float(empty)},
            "note": "agent_e2e's call with ~10% of versions re-sent later in the call, ~5% as two partial halves "
                    "(buffered, then ready), ~5% as Empty versions; headers in HBM, reset + fresh Bookie + call, "
                    f"median of {reps} after one untimed call"}


def run_multi(args, world, rank, pmc=(None, "not measured (--no-pmc)", None)):
    import torch
    import torch.distributed as dist
    import synth
    import corrosion_amd as ca
    from corrosion_amd.dist import distributed_apply_slots, exchange_records, slot_cap, verify_sites
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    # CORRO_BENCH_BACKEND=gloo rehearses the N>1 code path with several ranks on one GPU
    backend = os.environ.get("CORRO_BENCH_BACKEND", "nccl")
    if backend == "gloo":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    sdev = dev if backend == "nccl" else torch.device("cpu")   # where scalar reductions run
    strong = args.mode == "strong"
    if strong:
        G = args.changes or N_GLOBAL_C3
        lo, hi = rank * G // world, (rank + 1) * G // world
        npk = N_PK_C3
    else:
        G = (args.changes or N_CHANGES) * world
        lo, hi = rank * G // world, (rank + 1) * G // world
        npk = N_PK * world
    n_local = hi - lo
    eng = ca.MergeEngine({"t": ["a", "b", "c", "d"]}, capacity_hint=rank_capacity(n_local, G, npk, world), device=local)
    eng.register_sites(synth.site_ids(N_ACTORS, 1))
    verify_sites(eng)
    # rank r holds the global batch's slice r (rank-major = application order)
    batch = synth.uniform_batch_torch(n_local, N_ACTORS, npk, N_COLS, seed=synth.config_seed(3) + rank, device=dev,
                                      offset=lo, global_n=G)
    torch.cuda.synchronize()

    def barrier():
        dist.barrier()
        torch.cuda.synchronize()

    ex_ms = []
    # one slot size on every rank (equal all-to-all splits): from the largest rank's batch
    nmax = torch.tensor([n_local], device=sdev, dtype=torch.int64)
    dist.all_reduce(nmax, op=dist.ReduceOp.MAX)
    cap = slot_cap(int(nmax.item()), world)
    overflows = []

    def step():
        # stream-ordered: partition -> counts + slots all-to-all -> merge from the received slots
        # (corro_apply_slots: no unpack pass), all queued on the engine's stream (no host wait between
        # partition and merge)
        eng.reset()
        overflows.append(distributed_apply_slots(eng, batch, cap))

    def exchange_only():
        # the exact-size exchange alone (for exchange_ms and the owner-routed batch)
        t0 = time.perf_counter()
        recs, rb, counts, _ = eng.partition_packed(batch, world)
        got, _rc = exchange_records(recs, rb, counts)
        mine = eng.unpack_records(got, rb)
        torch.cuda.synchronize()
        ex_ms.append((time.perf_counter() - t0) * 1e3)
        return mine

    for _ in range(args.warmup):
        step()
    barrier()
    overflows.clear()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier()
    dt = time.perf_counter() - t0
    for _ in range(max(1, args.steps // 2)):
        mine = exchange_only()
    barrier()
    # owner-routed: the received batch IS this rank's owner-routed ingest; merge it alone
    prep = eng.prepare(mine)
    eng.reset()
    eng.apply_prepared(prep)
    barrier()
    t1 = time.perf_counter()
    for _ in range(args.steps):
        eng.reset()
        eng.apply_prepared(prep)
    barrier()
    dt_own = time.perf_counter() - t1
    stats = torch.tensor([dt, dt_own, sum(ex_ms) / max(1, len(ex_ms))], device=sdev, dtype=torch.float64)
    dist.all_reduce(stats, op=dist.ReduceOp.MAX)
    dt, dt_own, exm = (float(x) for x in stats.tolist())
    cells_t = torch.tensor([eng.count()], device=sdev, dtype=torch.int64)
    dist.all_reduce(cells_t, op=dist.ReduceOp.SUM)
    cells = int(cells_t.item())
    if rank == 0:
        # roofline of the whole step over the node: the SURVEY §8(d) algorithmic bytes of the merge
        # (48 B per change + 48 B per output cell) plus the exchange's 48 B x (N-1)/N per change
        # (strong mode: the packed records that leave their rank), against N x the HBM peak
        moved = ALG_BYTES_PER_CHANGE * G * (world - 1) / world
        alg = ALG_BYTES_PER_CHANGE * G + ALG_BYTES_PER_CELL * cells + moved
        achieved = alg / (dt / args.steps) / 1e9
        roof = {"bound": "hbm", "kernel": "step: slot partition + two equal-split all-to-alls + unpack + mapped merge, all ranks",
                "achieved": achieved, "peak": HBM_PEAK_GBS * world, "unit": "GB/s",
                "frac": achieved / (HBM_PEAK_GBS * world),
                "traffic": pmc[0] * world if pmc[0] else None,
                "traffic_per_rank": pmc[0],
                "traffic_source": (pmc[1] + "; per rank: rank 0's slice through the slot partition, unpack and "
                                   "mapped merge on one GPU (RCCL's copies excluded), x N for the node")
                if pmc[0] else pmc[1],
                "traffic_ratio": (pmc[0] * world / alg) if pmc[0] else None,
                "traffic_by_kernel_per_rank": ({k: {"fetch": round(v["fetch"]), "write": round(v["write"])}
                                                for k, v in sorted(pmc[2].items())} if pmc[2] else None),
                "alg_bytes_per_step": alg, "exchange_bytes_per_step": moved, "cells": cells}
        cpu = None if args.no_cpu_baseline else cpu_baseline_sample(npk)
        line = {
            "metric": METRIC,
            "value": G / dt * args.steps,
            "unit": "merged column-changes/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "int64",
            "data": "synthetic (seeded, generated in HBM)",
            "config": {"workload": ("config 3: 2^29 global column-changes (pk space 2^25, 1000 actors, 4 INTEGER cols, "
                                    "cl=1) arriving rank-major; per step: pk-hash partition into 48-B records + one "
                                    "all-to-all-v + unpack + merge of the owned rows") if strong else
                                   ("64M column-changes per GPU arriving on every GPU; per step: partition + one "
                                    "all-to-all-v + merge"),
                       "total_changes": G, "changes_per_gpu": n_local,
                       "parallelism": f"pk-hash x{world}, {backend} all-to-all"},
            "roofline": roof,
            "cpu_baseline": cpu,
            "exchange_ms": exm,
            "exchange": {"form": "stream-ordered slots: partition into fixed slots of cap records per destination, "
                                 "counts + slots in two equal-split all-to-alls on the engine's stream, mapped merge "
                                 "skipping the padding; no host wait between partition and merge",
                         "slot_cap": cap, "slot_padding": cap * world / max(1, n_local) - 1.0,
                         "overflowed_steps": int(sum(1 for o in overflows if o)),
                         "exchange_ms_note": "exchange_ms = the exact-size exchange timed alone (partition + "
                                             "counts + all-to-all-v + unpack, host-synchronised)"},
            "owner_routed": {"value": G / dt_own * args.steps, "ms_per_step": dt_own / args.steps * 1e3,
                             "note": "each rank merges only its own rows (the received batch), no collective"},
        }
        print(json.dumps(line), flush=True)
    eng.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
