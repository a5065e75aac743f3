"""Node-level multi-GPU merge: one process per GPU, rows sharded by pk hash.

Ingest on every rank: stable partition by owner rank into whole packed records (HIP kernel,
corro_partition_packed: 48 B per INTEGER change, the §8(d) record; corro_partition_var for tables
with interned pks or long values: 80-B records routed by the canonical pk bytes plus a second stream
of the pk / value bytes, re-keyed on the receiving engine) -> ONE all-to-all-v of records
(torch.distributed: RCCL over xGMI on the GPU box, gloo in CPU rehearsals) after one all-to-all of
the per-rank counts -> the received records, concatenated by source rank, unpacked to the SoA batch
(corro_unpack_records) -> local merge. Concatenation by source rank preserves every row's
application order when the global batch is rank-major. No further communication: rows merge
independently; per-site crsql_db_versions maxima reduce with one tiny all-reduce(max) when asked.

Site ordinals are per-engine, so the exchange is only meaningful between engines whose site tables
are identical (same 16-byte ids at the same ordinals): `verify_sites` all-gathers a digest of the
table and raises when a rank differs.
"""
import hashlib

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


def _counts_exchange(counts, dev, group):
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    send = torch.tensor(counts, dtype=torch.int64, device=dev)
    recv = torch.empty(world, dtype=torch.int64, device=dev)
    dist.all_to_all_single(recv, send, group=group)
    return [int(c) for c in recv.tolist()]


def exchange(parts, counts, group=None):
    """All-to-all-v of a rank-partitioned SoA batch, one collective per field (kept for batches a
    caller partitioned itself). `parts`: dict of 1-D tensors grouped by destination rank; `counts`:
    per-destination sizes. Returns the received dict (source-rank order)."""
    import torch
    import torch.distributed as dist
    dev = next(iter(parts.values())).device
    if dev.type == "cuda" and dist.get_backend(group) == "gloo":
        # gloo has no device all-to-all: stage through host memory (rehearsals on a 1-GPU box)
        got = exchange({k: v.cpu() for k, v in parts.items()}, counts, group)
        return {k: v.to(dev) for k, v in got.items()}
    out_splits = _counts_exchange(counts, dev, group)
    in_splits = [int(c) for c in counts]
    total = sum(out_splits)
    out = {}
    for k, a in parts.items():
        b = torch.empty(total, dtype=a.dtype, device=dev)
        dist.all_to_all_single(b, a, out_splits, in_splits, group=group)
        out[k] = b
    return out


def exchange_records(recs, rec_bytes, counts, group=None):
    """ONE all-to-all-v of packed records (uint8 tensor, grouped by destination rank, `counts`
    records each). Returns (received uint8 tensor in source-rank order, received counts)."""
    import torch
    import torch.distributed as dist
    dev = recs.device
    if dev.type == "cuda" and dist.get_backend(group) == "gloo":
        got, rc = exchange_records(recs.cpu(), rec_bytes, counts, group)
        return got.to(dev), rc
    rcounts = _counts_exchange(counts, dev, group)
    out = torch.empty(sum(rcounts) * rec_bytes, dtype=torch.uint8, device=dev)
    dist.all_to_all_single(out, recs, [c * rec_bytes for c in rcounts], [int(c) * rec_bytes for c in counts],
                           group=group)
    return out, rcounts


def exchange_var(recs, var, counts, vcounts, group=None):
    """The every-table exchange: the per-rank (records, bytes) sizes in one small all-to-all, then
    one all-to-all-v of 80-B records and one of their variable-length bytes. Returns (records,
    bytes, per-source record counts, per-source byte counts)."""
    import torch
    import torch.distributed as dist
    dev = recs.device
    if dev.type == "cuda" and dist.get_backend(group) == "gloo":
        r, v, rc, rv = exchange_var(recs.cpu(), var.cpu(), counts, vcounts, group)
        return r.to(dev), v.to(dev), rc, rv
    world = dist.get_world_size(group)
    send = torch.tensor([x for pair in zip(counts, vcounts) for x in pair], dtype=torch.int64, device=dev)
    got = torch.empty(2 * world, dtype=torch.int64, device=dev)
    dist.all_to_all_single(got, send, group=group)
    g = [int(x) for x in got.tolist()]
    rcounts, rvar = g[0::2], g[1::2]
    out = torch.empty(sum(rcounts) * 80, dtype=torch.uint8, device=dev)
    dist.all_to_all_single(out, recs, [c * 80 for c in rcounts], [int(c) * 80 for c in counts], group=group)
    vout = torch.empty(sum(rvar), dtype=torch.uint8, device=dev)
    dist.all_to_all_single(vout, var.contiguous(), rvar, [int(c) for c in vcounts], group=group)
    return out, vout, rcounts, rvar


def slot_cap(n_max, world):
    """Records per (source, destination) slot of the stream-ordered exchange: the even share of the
    largest rank's batch plus 8 standard deviations of a uniform hash split and a small floor, so a
    slot overflows only under skew (then the exchange repeats with exact sizes)."""
    share = n_max / world
    return int(share + 8.0 * share ** 0.5 + 256)


FAILED = -(1 << 63)  # a slot count with bit 63 set: the sender's batch failed (partition.hip's mark)


def _local(err, fn, *args, **kw):
    """Run one rank-local step of a multi-rank call unless an earlier step of this rank failed.
    Returns (result or None, the first error). A rank-local CorroError must not leave this rank
    outside the collectives its peers are about to enter (they would block in them, or see the
    connection drop): the caller goes on with empty contributions and reports the error in the
    call's last all-reduce, after which every rank raises (util.rs:849-855: the whole call fails)."""
    from ._lib import CorroError
    if err is not None:
        return None, err
    try:
        return fn(*args, **kw), None
    except CorroError as e:
        return None, e


def _raise_if_failed(err, nerr, world):
    """Every rank raises when any rank failed: its own error, or one naming the peers'."""
    from ._lib import CorroError
    if err is not None:
        raise err
    if nerr:
        raise CorroError(-3, f"multi-rank apply failed on {nerr} of {world} rank(s); this rank's own steps "
                             "succeeded (rows it merged stay merged: re-applying the same changes is a no-op)")


def _stream_ctx(engine, dev):
    import contextlib
    import torch
    return torch.cuda.stream(engine.stream()) if dev.type == "cuda" else contextlib.nullcontext()


def distributed_apply_slots(engine, batch, cap, group=None, impact=False):
    """The stream-ordered form of distributed_apply for INTEGER batches: partition into fixed slots of
    `cap` 48-B records per destination (slot_cap; the same cap on every rank), the per-slot counts and
    the slots in two all-to-alls with EQUAL splits, and the receiver's merge straight from the received
    slots (corro_apply_slots: its histogram and scatter read the records themselves -- no unpack pass)
    -- every step queued on the engine's stream (the collectives run under
    torch.cuda.stream(engine.stream())), so no host wait separates partition, exchange and merge.
    impact=True (process_multiple_changes always asks for crsql_rows_impacted(), util.rs:1247): the
    receiver's flags come out at slot positions, go back to their senders with a third equal-split
    all-to-all on the same stream, and the partition's permutation puts them in the caller's order
    (corro_slots_flags_back) -- still no host wait.
    A rank whose incoming slot overflowed merges nothing in that pass; after it, one tiny all-reduce
    tells every rank, and the exact-size exchange (distributed_apply) repeats for those ranks only.
    Failure (round 6): a rank whose partition, merge or flag pass raises still takes part in every
    collective of the call -- its counts marked failed (bit 63, so its receivers merge nothing from it),
    zero flags -- and the same all-reduce that carries the overflow count carries an error count, after
    which EVERY rank raises (the reference fails the whole call, util.rs:849-855), none blocks.
    Returns the number of ranks that overflowed (0 in the common case), and with impact=True the flags
    (uint8 CUDA tensor, this rank's changes in its own order) as a second value."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    if world == 1:
        imp = engine.apply(batch, impact=impact)
        return (0, imp) if impact else 0
    n = int(batch["pk"].shape[0])
    dev = batch["pk"].device
    cuda = dev.type == "cuda"
    if cuda:
        engine.stream().wait_stream(torch.cuda.current_stream())  # the batch's producer (device-side wait)
    gloo = dist.get_backend(group) == "gloo"

    def a2a(dst, src):
        if gloo and cuda:  # (no device all-to-all in gloo: rehearsals stage through host memory)
            h = torch.empty(src.numel(), dtype=src.dtype)
            dist.all_to_all_single(h, src.cpu(), group=group)
            dst.copy_(h.to(dst.device))
        else:
            dist.all_to_all_single(dst, src, group=group)

    err = None
    with _stream_ctx(engine, dev):
        perm = torch.empty(world * cap, dtype=torch.int32, device=dev) if impact else None
        got_p, err = _local(err, engine.partition_slots, batch, world, cap, perm=perm)
        if got_p is None:  # (failed here: empty slots, every count marked failed)
            recs = torch.zeros(world * cap * 48, dtype=torch.uint8, device=dev)
            cnt = torch.full((world,), FAILED, dtype=torch.int64, device=dev)
        else:
            recs, cnt = got_p
        rcnt = torch.empty_like(cnt)
        a2a(rcnt, cnt)
        got = torch.empty_like(recs)
        a2a(got, recs)
        res, err = _local(err, engine.apply_slots, got, world, cap, rcnt, impact=impact)
        imp_slots, over = res if res is not None else (None, None)
        if over is None:
            over = torch.zeros(1, dtype=torch.int32, device=dev)
        flags = None
        if impact:
            if imp_slots is None:
                imp_slots = torch.zeros(world * cap, dtype=torch.uint8, device=dev)
            back = torch.empty_like(imp_slots)
            a2a(back, imp_slots)
            flags, err = _local(err, engine.slots_flags_back, back, world, cap, cnt, perm, n)
        over = over.to(torch.int64).reshape(1)  # (on the engine's stream, where the apply wrote it)
    if cuda:
        torch.cuda.current_stream().wait_stream(engine.stream())  # (the caller reads `over`, the flags, the state)
    # one all-reduce: [ranks that overflowed, ranks that failed]
    tot = torch.cat([over.cpu() if (gloo or not cuda) else over,
                     torch.tensor([1 if err is not None else 0], dtype=torch.int64,
                                  device="cpu" if (gloo or not cuda) else dev)])
    dist.all_reduce(tot, op=dist.ReduceOp.SUM, group=group)
    nover, nerr = (int(x) for x in tot.tolist())
    _raise_if_failed(err, nerr, world)
    if nover:
        mine = int(over.item())
        res, err = _local(None, engine.partition_packed, batch, world, with_perm=impact)
        if res is None:
            recs2, rb, counts, perm2 = torch.zeros(0, dtype=torch.uint8, device=dev), 48, [0] * world, None
        else:
            recs2, rb, counts, perm2 = res
        got2, rc2 = exchange_records(recs2, rb, counts, group)
        imp2 = None
        if mine:
            unp, err = _local(err, engine.unpack_records, got2, rb)
            if unp is not None:
                imp2, err = _local(err, engine.apply, unp, impact=impact)
        if impact:  # every rank takes part in the flags' way back (the overflowed ones send real flags)
            send = imp2[:sum(rc2)].contiguous() if imp2 is not None else torch.zeros(sum(rc2), dtype=torch.uint8,
                                                                                     device=dev)
            back2 = torch.empty(sum(counts), dtype=torch.uint8, device=dev)
            if gloo and cuda:
                b2 = torch.empty(sum(counts), dtype=torch.uint8)
                dist.all_to_all_single(b2, send.cpu(), [int(c) for c in counts], rc2, group=group)
                back2 = b2.to(dev)
            else:
                dist.all_to_all_single(back2, send, [int(c) for c in counts], rc2, group=group)
            # flags from destinations that overflowed replace the slot pass's (which applied nothing there)
            ov = over.cpu() if (gloo or not cuda) else over
            allov = [torch.zeros_like(ov) for _ in range(world)]
            dist.all_gather(allov, ov, group=group)
            dst_over = torch.cat([x.cpu() for x in allov]).tolist()
            if err is None and perm2 is not None:
                start = 0
                p2 = perm2.long()
                for d, c in enumerate(counts):
                    if dst_over[d]:
                        flags[p2[start:start + int(c)]] = back2[start:start + int(c)]
                    start += int(c)
        e2 = torch.tensor([1 if err is not None else 0], dtype=torch.int64,
                          device="cpu" if (gloo or not cuda) else dev)
        dist.all_reduce(e2, op=dist.ReduceOp.SUM, group=group)
        _raise_if_failed(err, int(e2.item()), world)
    return (nover, flags) if impact else nover


def site_digest(engine):
    """sha256 of the engine's site table (16-byte ids in ordinal order)."""
    return hashlib.sha256(b"".join(engine.site_ids())).digest()


def verify_sites(engine, group=None):
    """Raise unless every rank's engine holds the same site table (ids at the same ordinals): the
    packed records carry site ordinals, which would otherwise land under the wrong site id and
    break the merge-equal-values tie-break."""
    import torch.distributed as dist
    mine = site_digest(engine)
    got = [None] * dist.get_world_size(group)
    dist.all_gather_object(got, mine, group=group)
    bad = [r for r, d in enumerate(got) if d != mine]
    if bad:
        raise RuntimeError(f"site tables differ between ranks {bad} and this one: register the same site ids "
                           "in the same order on every rank before exchanging changes")


def distributed_apply(engine, batch, group=None, impact=False, verify=True):
    """Partition by owner rank into packed records, exchange them with one all-to-all, merge the
    owned rows into this rank's engine. With impact=True returns the crsql_rows_impacted() growth
    of THIS rank's input changes, in the caller's order (a second, 1-byte-per-change all-to-all
    sends every flag back to its sender, and the partition's permutation restores the order).
    A rank-local failure (partition, unpack, merge) still joins every collective with empty
    contributions; one all-reduce of an error count at the end makes every rank raise."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    if world == 1:
        return engine.apply(batch, impact=impact)
    if verify:
        n_sites = engine.site_count()
        if getattr(engine, "_sites_verified", None) != n_sites:
            verify_sites(engine, group)
            engine._sites_verified = n_sites
    dev = batch["pk"].device
    err = None
    n_in = int(batch["pk"].shape[0])
    if "val_data" in batch or engine.interned:
        # interned pks (routed and re-keyed by their canonical bytes) or long values: records + bytes
        res, err = _local(err, engine.partition_var, batch, world, with_perm=impact)
        if res is None:
            z = torch.zeros(0, dtype=torch.uint8, device=dev)
            recs, var, counts, vcounts, perm = z, z, [0] * world, [0] * world, None
        else:
            recs, var, counts, vcounts, perm = res
        got, gvar, rcounts, rvar = exchange_var(recs, var, counts, vcounts, group)
        mine, err = _local(err, engine.unpack_var, got, gvar, rcounts, rvar)
    else:
        res, err = _local(err, engine.partition_packed, batch, world, with_perm=impact)
        if res is None:
            recs, rb, counts, perm = torch.zeros(0, dtype=torch.uint8, device=dev), 48, [0] * world, None
        else:
            recs, rb, counts, perm = res
        got, rcounts = exchange_records(recs, rb, counts, group)
        mine, err = _local(err, engine.unpack_records, got, rb)
    imp = None
    if mine is not None:
        imp, err = _local(err, engine.apply, mine, impact=impact)
    out = None
    if impact:
        # flags back to the senders (reverse split sizes), then into the caller's order
        send = imp[:sum(rcounts)].contiguous() if imp is not None else torch.zeros(sum(rcounts), dtype=torch.uint8,
                                                                                   device=dev)
        back = torch.empty(sum(counts), dtype=torch.uint8, device=dev)
        if dev.type == "cuda" and dist.get_backend(group) == "gloo":
            b2 = torch.empty(sum(counts), dtype=torch.uint8)
            dist.all_to_all_single(b2, send.cpu(), [int(c) for c in counts], rcounts, group=group)
            back = b2.to(dev)
        else:
            dist.all_to_all_single(back, send, [int(c) for c in counts], rcounts, group=group)
        if perm is not None:
            out = torch.zeros(n_in, dtype=torch.uint8, device=dev)
            out[perm.long()] = back
    cpu_red = dev.type != "cuda" or dist.get_backend(group) == "gloo"
    e = torch.tensor([1 if err is not None else 0], dtype=torch.int64, device="cpu" if cpu_red else dev)
    dist.all_reduce(e, op=dist.ReduceOp.SUM, group=group)
    _raise_if_failed(err, int(e.item()), world)
    return out
