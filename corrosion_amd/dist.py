"""Node-level multi-GPU merge: one process per GPU, rows sharded by pk hash.

Ingest on every rank: stable partition by owner rank (HIP kernel, corro_partition_ranks) ->
one all-to-all-v exchange per SoA field (torch.distributed, RCCL over xGMI on the GPU box) ->
concatenation by source rank (preserves every row's application order when the global batch is
rank-major) -> local merge. No further communication: rows merge independently; per-site
crsql_db_versions maxima reduce with one tiny all-reduce(max) when asked.
"""
import numpy as np

MASK64 = (1 << 64) - 1


def _mix64_np(x):
    x = x.astype(np.uint64)
    with np.errstate(over="ignore"):
        x ^= x >> np.uint64(33)
        x *= np.uint64(0xFF51AFD7ED558CCD)
        x ^= x >> np.uint64(33)
        x *= np.uint64(0xC4CEB9FE1A85EC53)
        x ^= x >> np.uint64(33)
    return x


def rank_of_np(table_cid, pk, nranks):
    """Host mirror of rank_of() in csrc/partition.hip (owner rank of a row)."""
    table = (np.asarray(table_cid, np.uint64) >> np.uint64(16))
    with np.errstate(over="ignore"):
        h = _mix64_np(np.asarray(pk, np.uint64) + np.uint64(0x9E3779B97F4A7C15) * (table + np.uint64(1)))
    return ((h & np.uint64(0xFFFFFFFF)) % np.uint64(nranks)).astype(np.int64)


def exchange(parts, counts, group=None):
    """All-to-all-v of a rank-partitioned batch. `parts`: dict of 1-D tensors grouped by
    destination rank; `counts`: per-destination sizes. Returns the received dict (source-rank
    order) — works on CUDA tensors with nccl (RCCL) and on CPU tensors with gloo."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    dev = next(iter(parts.values())).device
    if dev.type == "cuda" and dist.get_backend(group) == "gloo":
        # gloo has no device all-to-all: stage through host memory (rehearsals on a 1-GPU box)
        got = exchange({k: v.cpu() for k, v in parts.items()}, counts, group)
        return {k: v.to(dev) for k, v in got.items()}
    send = torch.tensor(counts, dtype=torch.int64, device=dev)
    recv = torch.empty(world, dtype=torch.int64, device=dev)
    dist.all_to_all_single(recv, send, group=group)
    in_splits = [int(c) for c in counts]
    out_splits = [int(c) for c in recv.tolist()]
    total = sum(out_splits)
    out = {}
    for k, a in parts.items():
        b = torch.empty(total, dtype=a.dtype, device=dev)
        dist.all_to_all_single(b, a, out_splits, in_splits, group=group)
        out[k] = b
    return out


def distributed_apply(engine, batch, group=None, impact=False):
    """Partition by owner rank, exchange, merge the owned rows into this rank's engine."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    if world == 1:
        return engine.apply(batch, impact=impact), None
    parts, counts = engine.partition(batch, world)
    mine = exchange(parts, counts, group)
    return engine.apply(mine, impact=impact), mine
