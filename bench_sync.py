"""Config-4 benchmark: batched SyncStateV1 need diff (compute_available_needs) on MI355X.

BASELINE.json configs[3]: 1M node-pair sync states, 64 sparse actors per pair from a 100k-actor
universe -> 64M (pair, actor) entries, generated in HBM (synth.sync_entries_torch). One step =
corro_compute_needs count pass + device offset scan + fill pass (default), or with --one-pass
corro_compute_needs_onepass. Algorithmic bytes:
16 B per input range (ours.need, theirs.need, partial seq ranges) + 16 B per head pair + 8 B per
partial version + 16 B per output range. Prints one JSON line.

--gpus N (SURVEY §8(e) last bullet): node pairs are independent, so the 1M pairs are sharded
contiguously over N ranks (one process per GPU, launched by this script unless WORLD_SIZE is set)
with no exchange on the data path: each rank diffs its own pairs and keeps its outputs (strong
scaling; `value` = all pairs / the slowest rank's step, barrier + max over ranks).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
HBM_PEAK_GBS = 8000.0


def _host_cut(ent_dev, n):
    """The first n entries' CSR arrays copied to host memory (offsets stay absolute)."""
    import numpy as np
    cut = {}
    for k in ("their_head", "our_head"):
        cut[k] = ent_dev[k][:n].cpu().numpy()
    for side in ("tn", "on", "tp", "op"):
        off = ent_dev[f"{side}_off"][: n + 1].cpu().numpy()
        cut[f"{side}_off"] = off
        m = int(off[-1])
        if side in ("tn", "on"):
            cut[f"{side}_start"] = ent_dev[f"{side}_start"][:m].cpu().numpy()
            cut[f"{side}_end"] = ent_dev[f"{side}_end"][:m].cpu().numpy()
        else:
            cut[f"{side}_ver"] = ent_dev[f"{side}_ver"][:m].cpu().numpy()
            so = ent_dev[f"{side}s_off"][: m + 1].cpu().numpy()
            cut[f"{side}s_off"] = so
            cut[f"{side}s_start"] = ent_dev[f"{side}s_start"][: int(so[-1])].cpu().numpy()
            cut[f"{side}s_end"] = ent_dev[f"{side}s_end"][: int(so[-1])].cpu().numpy()
    return {k: np.ascontiguousarray(v) for k, v in cut.items()}


def cpu_baseline(ent_dev, sample, threads=16):
    """oracle/ranges.c compute_available_needs (kind 'port'): every entry of the rank's workload on
    `threads` host threads (oracle.needs_parallel: 1 M-entry chunks, the C passes release the GIL),
    plus the 1-core rate on the first `sample` entries. `value` is the multi-thread rate."""
    from oracle import oracle as O
    E = int(ent_dev["their_head"].shape[0])
    full = _host_cut(ent_dev, E)
    t0 = time.perf_counter()
    O.needs_parallel(full, nthreads=threads)
    dt = time.perf_counter() - t0
    del full
    one = _host_cut(ent_dev, sample)
    t0 = time.perf_counter()
    O.needs(one)
    dt1 = time.perf_counter() - t0
    return {"value": E / dt, "unit": "entries/s", "cores": threads, "kind": "port",
            "sample": f"all {E} (pair, actor) entries of the workload, oracle/ranges.c count+fill passes on "
                      f"{threads} threads in {dt:.2f} s",
            "one_core": {"value": sample / dt1, "unit": "entries/s", "cores": 1,
                         "sample": f"first {sample} entries in {dt1:.2f} s"}}


def _packed_seq_total(res):
    """Seq ranges of a packed result, from the written need slots only."""
    import torch
    cnt = res["need_count"].to(torch.int64)
    T = int(cnt.sum())
    off = torch.zeros_like(cnt)
    off[1:] = torch.cumsum(cnt, 0)[:-1]
    slot = torch.repeat_interleave(res["need_off"] - off, cnt) + torch.arange(T, device=cnt.device)
    hi = res["range"].view(-1, 2)[slot, 1]
    return int(torch.where(res["kind"][slot] == 1, hi & 0xFFFFFF, 0).sum())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=1_000_000)
    ap.add_argument("--actors-per-pair", type=int, default=64)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--cpu-sample", type=int, default=200_000)
    ap.add_argument("--no-pmc", action="store_true", help="skip the live rocprofv3 traffic passes")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--mode", choices=("packed", "two-pass", "one-pass"), default="packed",
                    help="packed: corro_compute_needs_packed (one pass into bound-reserved slots, 16-B need "
                         "pairs); two-pass: corro_compute_needs count + fill; one-pass: "
                         "corro_compute_needs_onepass (decoupled look-back)")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        from bench import launch_ranks
        sys.exit(launch_ranks(args.gpus, __file__))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    PMC_RUNS = 3
    traffic = None
    if world == 1 and not args.pmc_child and not args.no_pmc:
        # HBM bytes per diff from rocprofv3 FETCH_SIZE / WRITE_SIZE passes over a child run of this
        # script doing PMC_RUNS diffs, before this process touches the GPU (bench.py's recipe)
        from bench import pmc_traffic_live
        child = [os.path.abspath(__file__), "--pmc-child", "--mode", args.mode, "--pairs", str(args.pairs),
                 "--actors-per-pair", str(args.actors_per_pair)]
        tb, note, per = pmc_traffic_live(0, applies=PMC_RUNS, child_cmd=child)
        if per:  # the need-diff kernels only (the child's data generation runs torch / rocPRIM kernels)
            per = {k: v for k, v in per.items() if k.startswith("k_needs") or k.startswith("k_scan")}
            tb = sum(v["fetch"] + v["write"] for v in per.values())
        traffic = {"bytes": tb, "source": note, "by_kernel": per}

    import torch
    import synth
    import corrosion_amd as ca
    from corrosion_amd.sync import _needs_device, _needs_device_1pass, _needs_device_packed
    run = {"packed": _needs_device_packed, "two-pass": _needs_device, "one-pass": _needs_device_1pass}[args.mode]

    dist = None
    local = 0
    if world > 1:
        import torch.distributed as dist
        backend = os.environ.get("CORRO_BENCH_BACKEND", "nccl")
        local = int(os.environ.get("LOCAL_RANK", str(rank))) % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    eng = ca.MergeEngine({"t": ["a"]}, capacity_hint=1024, device=local)
    pairs_local = (rank + 1) * args.pairs // world - rank * args.pairs // world
    ent = synth.sync_entries_torch(pairs_local, args.actors_per_pair, synth.config_seed(4) + 7919 * rank, device=dev)
    torch.cuda.synchronize()
    if args.pmc_child:  # exactly PMC_RUNS diffs, nothing else of ours
        for _ in range(PMC_RUNS):
            run(eng, ent)
        torch.cuda.synchronize()
        return
    eng.set_profiling(True)
    for _ in range(args.warmup):
        res = run(eng, ent)
    kt = kc = kf = 0.0
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = run(eng, ent)
        tm = eng.last_timings(apply_only=False)
        kc += tm["k_needs_count"]
        kf += tm["k_needs_fill"]
        kt += tm["k_needs_count"] + tm["k_needs_fill"]
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    dt = (time.perf_counter() - t0) / args.steps
    if dist is not None:
        x = torch.tensor([dt], dtype=torch.float64, device=dev if os.environ.get("CORRO_BENCH_BACKEND", "nccl") == "nccl"
                         else "cpu")
        dist.all_reduce(x, op=dist.ReduceOp.MAX)
        dt = float(x.item())
    kt /= args.steps
    kc /= args.steps
    kf /= args.steps
    E = int(ent["their_head"].shape[0])
    in_ranges = sum(int(ent[k].shape[0]) for k in ("tn_start", "on_start", "tps_start", "ops_start"))
    pvers = int(ent["tp_ver"].shape[0] + ent["op_ver"].shape[0])
    if args.mode == "packed":
        n_needs = int(res["need_count"].to(torch.int64).sum())
        n_seqs = _packed_seq_total(res)  # (from the written slots only: the padding holds garbage)
    else:
        n_needs, n_seqs = int(res["start"].shape[0]), int(res["s_start"].shape[0])
    out_ranges = n_needs + n_seqs
    alg = 16 * in_ranges + 16 * E + 8 * pvers + 16 * out_ranges
    achieved = alg / (kt * 1e-3) / 1e9
    line = {"metric": "SyncStateV1 need diff: node-pairs/s (config 4)", "value": args.pairs / dt,
            "unit": "node-pairs/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": dt * 1e3, "higher_is_better": True, "scaling": "strong" if world > 1 else "n/a",
            "dtype": "u64", "data": "synthetic (HBM)",
            "config": {"workload": "config 4", "pairs": args.pairs, "entries_rank0": E, "input_ranges_rank0": in_ranges,
                       "output_needs_rank0": n_needs, "output_seq_ranges_rank0": n_seqs, "mode": args.mode,
                       "parallelism": f"{world} rank(s), node pairs sharded, no exchange"},
            "entries_per_s": E * world / dt,
            "roofline": {"bound": "hbm", "kernel": {"packed": "k_needs_packed (one pass)", "two-pass": "k_needs (count + fill)",
                                                    "one-pass": "k_needs1 (one pass, look-back)"}[args.mode],
                         "achieved": achieved,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "traffic": traffic["bytes"] if traffic else None,
                         "traffic_ratio": (traffic["bytes"] / alg) if traffic and traffic["bytes"] else None,
                         "traffic_by_kernel": traffic["by_kernel"] if traffic else None,
                         "alg_bytes": alg,
                         "output_bytes": (17 * n_needs + 12 * E if args.mode == "packed" else 33 * n_needs + 32 * E)
                         + 16 * n_seqs,
                         "kernels_ms": kt, "count_pass_ms": kc, "fill_pass_ms": kf}}
    if rank == 0:
        if world == 1:
            line["cpu_baseline"] = cpu_baseline(ent, min(args.cpu_sample, E))
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
