"""Headline benchmark: merged column-changes/s of the batched crsql_changes merge on MI355X.

Workload = BASELINE.json configs[1]: 64M (2^26) column changes, 1 table with 4 INTEGER columns,
1000 actors, pk uniform in [1, 2^22], col_version uniform [1, 8], 1/8 of values from {0..7}
(value ties), cl = 1, 64 changes per version per actor. Synthetic data
generated directly in HBM. One step = one `process_multiple_changes`-sized apply of the whole
batch into an empty state (state reset + corro_apply_batch), inputs already resident in HBM.

Multi-GPU (torchrun, one process per GPU): rows are owned by pk hash
(corro_partition_ranks' rank_of), every row merges independently, so each rank merges the ~64M
changes of ITS rows with no collective on the data path (weak scaling: per-GPU work fixed; the
batch each rank holds is the owner-routed ingest of config 3, routed when it is built, outside the
timed region). `--exchange` instead times partition + RCCL all-to-all-v + merge per step for
batches that arrive mixed on every GPU (the ingest-exchange variant, reported in DESIGN.md §6).

Prints ONE JSON line (rank 0).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

N_CHANGES = 1 << 26
N_ACTORS = 1000
N_PK = 1 << 22
N_COLS = 4
ALG_BYTES_PER_CHANGE = 48  # pk 8, table_cid 4, col_version 8, db_version 8, cl 4, seq 4, site 4, value 8
ALG_BYTES_PER_CELL = 48
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: 8 TB/s spec


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
                            "sample": f"{n} changes of the config-2 distribution folded sequentially in {dt:.2f} s"}}


PIPELINE_KERNELS = ("k_hist", "k_colscan", "k_plan", "k_scatter", "k_merge_fast", "k_merge_gen", "k_merge_ovf")


def pmc_traffic_per_apply():
    """HBM bytes per apply from the committed rocprofv3 PMC passes (profiles/*_pmc_{FETCH,WRITE}_SIZE.csv,
    collected by scripts/gpu_prof.sh on this bench): sum over the pipeline kernels of
    2 x FETCH_SIZE (gfx950 reports half of wide coalesced reads, MI355X_MICROARCH.md §HBM) +
    WRITE_SIZE, in KiB -> bytes, averaged per dispatch. None when the files are absent."""
    import csv
    import glob
    from collections import defaultdict
    out = {}
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r[0-9][0-9]_pmc_{counter}.csv")))
        if not files:
            return None, None
        tot, disp = defaultdict(float), defaultdict(set)
        for r in csv.DictReader(open(files[-1])):
            name = r["Kernel_Name"]
            k = next((p for p in PIPELINE_KERNELS if p in name), None)
            if k and r["Counter_Name"] == counter:
                tot[k] += float(r["Counter_Value"])
                disp[k].add(r["Dispatch_Id"])
        out[counter] = sum(tot[k] / len(disp[k]) for k in tot)
        src = os.path.basename(files[-1])
    return (2 * out["FETCH_SIZE"] + out["WRITE_SIZE"]) * 1024.0, src


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--changes", type=int, default=N_CHANGES)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--exchange", action="store_true",
                    help="N>1: time partition + RCCL all-to-all + merge (batches arrive mixed on every GPU)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    import synth
    import corrosion_amd as ca

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # CORRO_BENCH_BACKEND=gloo rehearses the N>1 code path with several ranks on one GPU
    backend = os.environ.get("CORRO_BENCH_BACKEND", "nccl")
    if backend == "gloo":
        local = local % max(1, torch.cuda.device_count())
    if world > 1:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    sdev = dev if backend == "nccl" else torch.device("cpu")  # where scalar reductions run

    n = args.changes
    eng = ca.MergeEngine({"t": ["a", "b", "c", "d"]}, capacity_hint=n, device=local)
    sites = synth.site_ids(N_ACTORS, 1)
    eng.register_sites(sites)
    seed = synth.config_seed(2) + rank
    if world == 1 or args.exchange:
        batch = synth.uniform_batch_torch(n, N_ACTORS, N_PK * world, N_COLS, seed=seed, device=dev)
    else:
        # owner-routed ingest: keep this rank's rows out of `world` chunks of candidates drawn over
        # the whole node's pk space (untimed setup)
        own = []
        for c in range(world):
            cand = synth.uniform_batch_torch(n, N_ACTORS, N_PK * world, N_COLS, seed=seed * 1000 + c, device=dev)
            parts, counts = eng.partition(cand, world)
            lo = sum(counts[:rank])
            own.append({k: v[lo:lo + counts[rank]].clone() for k, v in parts.items()})
            del cand, parts
        batch = {k: torch.cat([o[k] for o in own]).contiguous() for k in own[0]}
        del own
        torch.cuda.empty_cache()
    n_local = int(batch["pk"].shape[0])
    torch.cuda.synchronize()
    eng.set_profiling(True)
    from corrosion_amd.dist import distributed_apply

    # the batch's C-ABI descriptor (device pointers and sizes) is built once: a Rust caller hands
    # the same struct over; every step still resets the state and runs the whole apply
    prep = eng.prepare(batch)

    def step():
        eng.reset()
        if world > 1 and args.exchange:
            distributed_apply(eng, batch)
        else:
            eng.apply_prepared(prep)

    for _ in range(args.warmup):
        step()
    cells = eng.count()

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    kern = {}
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        for k, v in eng.last_timings().items():
            kern[k] = kern.get(k, 0.0) + v
    barrier()
    dt = time.perf_counter() - t0
    total = n_local * world if args.exchange else n_local
    if world > 1:
        t = torch.tensor([dt], device=sdev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        if not args.exchange:
            tot = torch.tensor([n_local], device=sdev, dtype=torch.int64)
            dist.all_reduce(tot)
            total = int(tot.item())
    kern = {k: v / args.steps for k, v in kern.items()}
    pipe_ms = sum(v for k, v in kern.items())
    dominant = max(kern, key=kern.get)
    # per-GPU algorithmic bytes of one merge (with --exchange the merged slice is the received one,
    # of the same expected size as the local batch)
    alg_bytes = ALG_BYTES_PER_CHANGE * n_local + ALG_BYTES_PER_CELL * cells
    achieved = alg_bytes / (pipe_ms * 1e-3) / 1e9

    if rank == 0:
        traffic, traffic_src = pmc_traffic_per_apply()
        cpu = None if args.no_cpu_baseline or world > 1 else cpu_baseline(batch)
        line = {
            "metric": "merged column-changes/sec (node) at 1/2/4/8 GPUs + % of HBM BW roofline",
            "value": total / dt * args.steps,
            "unit": "merged column-changes/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int64",
            "data": "synthetic (seeded, generated in HBM)",
            "config": {"workload": "config 2: 64M column-changes, 1 table x 4 INTEGER cols, 1000 actors, "
                                   "uniform pk in [1,2^22] per GPU, cl=1, bucket merge"
                                   + ("" if world == 1 else
                                      ("; + pk-hash partition and RCCL all-to-all per step" if args.exchange else
                                       "; rows owned by pk hash, each rank merges its own rows (no data-path collective)")),
                       "changes_per_gpu": n_local, "total_changes": total, "cells_per_gpu": int(cells),
                       "parallelism": f"pk-hash x{world}" + (" + all-to-all" if world > 1 and args.exchange else "")},
            "roofline": {"bound": "hbm", "kernel": "apply pipeline: " + "+".join(k for k in kern if kern[k] > 0),
                         "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                         "alg_bytes_per_apply": alg_bytes, "pipeline_ms": pipe_ms,
                         "kernels_ms": kern, "dominant": dominant},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
