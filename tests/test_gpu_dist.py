"""Two ranks on one GPU box: device pk-hash partition (HIP) + all-to-all exchange (gloo through host
memory here; RCCL on a multi-GPU node) + per-rank device merge. The union of the rank states must
equal the single-engine merge of the whole batch, bit for bit, and that merge the oracle's
sequential fold (rows, impact flags, db_versions)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import synth
from tests._util import rows_to_tuples

pytestmark = pytest.mark.gpu
N, SEED, NT = 40000, 95, 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _to_dev(b):
    import torch
    return {k: torch.from_numpy(np.ascontiguousarray(v).view(
        np.int64 if v.dtype == np.uint64 else (np.int32 if v.dtype == np.uint32 else v.dtype))).cuda()
        for k, v in b.items()}


def _worker(rank, world, port, outdir):
    import torch.distributed as dist
    import corrosion_amd as ca
    from corrosion_amd.dist import distributed_apply, rank_of_np
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sites = synth.site_ids(8, SEED)
    full = synth.adversarial_batch(N, 8, NT, 500, SEED)
    lo, hi = rank * N // world, (rank + 1) * N // world
    eng = ca.MergeEngine(synth.adversarial_schema(NT), capacity_hint=N, device=0)
    eng.register_sites(sites)
    imp = distributed_apply(eng, _to_dev({k: v[lo:hi] for k, v in full.items()}), impact=True)
    np.save(os.path.join(outdir, f"imp{rank}.npy"), imp.cpu().numpy())
    rows = eng.export()
    assert (rank_of_np(rows["table_cid"], rows["pk"], world) == rank).all()
    np.save(os.path.join(outdir, f"rows{rank}.npy"), np.array(rows_to_tuples(rows, with_ts=True), dtype=object),
            allow_pickle=True)
    eng.close()
    dist.destroy_process_group()


def test_two_rank_device_merge_equals_single_engine(tmp_path):
    import corrosion_amd as ca
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    got = []
    for r in range(world):
        got += [tuple(x) for x in np.load(tmp_path / f"rows{r}.npy", allow_pickle=True)]
    from oracle import oracle as O
    e = ca.MergeEngine(synth.adversarial_schema(NT), capacity_hint=N)
    e.register_sites(synth.site_ids(8, SEED))
    batch = synth.adversarial_batch(N, 8, NT, 500, SEED)
    want_imp = e.apply(batch, impact=True)
    assert sorted(got) == rows_to_tuples(e.export(), with_ts=True)
    # per-change impacts come back to each sender in its own order (reverse all-to-all + permutation)
    got_imp = np.concatenate([np.load(tmp_path / f"imp{r}.npy") for r in range(world)])
    assert np.array_equal(got_imp, want_imp)
    # and the single engine (so the union of the ranks) against the oracle's sequential fold
    f = O.Fold(synth.site_ids(8, SEED))
    assert np.array_equal(want_imp, f.apply(batch))
    assert O.rows_diff(e.export(), f.export()) is None


def _sites_worker(rank, world, port, outdir):
    import torch.distributed as dist
    import corrosion_amd as ca
    from corrosion_amd.dist import verify_sites
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    eng = ca.MergeEngine(synth.adversarial_schema(NT), capacity_hint=1 << 12, device=0)
    sites = synth.site_ids(4, SEED)
    eng.register_sites(sites if rank == 0 else sites[::-1])  # same ids, different ordinals
    try:
        verify_sites(eng)
        ok = "verified"
    except RuntimeError:
        ok = "refused"
    open(os.path.join(outdir, f"sites{rank}.txt"), "w").write(ok)
    eng.close()
    dist.destroy_process_group()


def test_exchange_refuses_mismatched_site_tables(tmp_path):
    world = 2
    mp.spawn(_sites_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    assert [open(tmp_path / f"sites{r}.txt").read() for r in range(world)] == ["refused", "refused"]


# ---- every table: interned pks (testsblob, wide) and long values over the exchange ----------------
NV, SEEDV = 9000, 17


def _pk_batch(eng, rows):
    """rows of tests.test_gpu_pk._changes -> a host batch keyed on THIS engine (interned ids are per
    engine: the exchange must re-key them from the canonical bytes)."""
    from tests.test_gpu_pk import INTERNED, SCHEMA
    from tests._util import encode_values
    from corrosion_amd.wire import unpack_int_pk
    tix = {t: i for i, t in enumerate(SCHEMA)}
    keys = np.zeros(len(rows), np.uint64)
    for t in SCHEMA:
        idx = [j for j, r in enumerate(rows) if r[0] == t]
        if not idx:
            continue
        if t in INTERNED:
            keys[idx] = eng.pk_keys(t, [rows[j][1] for j in idx])
        else:
            keys[idx] = [unpack_int_pk(rows[j][1]) & 0xFFFFFFFFFFFFFFFF for j in idx]
    b = {"pk": keys,
         "table_cid": np.array([(tix[r[0]] << 16) | r[2] for r in rows], np.uint32),
         "col_version": np.array([r[4] for r in rows], np.int64),
         "db_version": np.array([r[5] for r in rows], np.int64),
         "site": np.array([r[6] for r in rows], np.uint32),
         "cl": np.array([r[7] for r in rows], np.uint32),
         "seq": np.array([r[8] % 100 for r in rows], np.uint32),
         "ts": np.array([r[8] for r in rows], np.uint64)}
    b.update(encode_values([r[3] for r in rows]))
    return b


def _canon_rows(eng):
    """the state as comparable tuples: interned row keys by their canonical packed pk, long values
    by their bytes"""
    from tests.test_gpu_pk import INTERNED, SCHEMA
    rows = eng.export()
    tups = rows_to_tuples(rows, with_ts=True)
    out = []
    names = list(SCHEMA)
    for t in tups:
        name = names[t[0]]
        pk = eng.pk_bytes(name, [t[1]])[0] if name in INTERNED else t[1]
        out.append((t[0], pk) + t[2:])
    return sorted(out, key=repr)


def _var_worker(rank, world, port, outdir):
    import pickle
    import torch
    import torch.distributed as dist
    import corrosion_amd as ca
    from corrosion_amd.dist import distributed_apply
    from tests.test_gpu_pk import INTERNED, SCHEMA, _changes
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(SEEDV)
    rows = _changes(rng, NV, 6)
    lo, hi = rank * NV // world, (rank + 1) * NV // world
    eng = ca.MergeEngine(SCHEMA, capacity_hint=NV, device=0, interned=INTERNED)
    eng.register_sites(synth.site_ids(6, 3))
    if rank == 1:  # a different interning order than rank 0: the shipped bytes must re-key rows
        eng.pk_keys("wide", [r[1] for r in reversed(rows) if r[0] == "wide"][:40])
    b = _pk_batch(eng, rows[lo:hi])
    dev = {}
    for k, v in b.items():
        v = np.ascontiguousarray(v)
        dev[k] = torch.from_numpy(v.view(np.int64) if v.dtype == np.uint64 else
                                  (v.view(np.int32) if v.dtype == np.uint32 else v)).cuda()
    imp = distributed_apply(eng, dev, impact=True)
    np.save(os.path.join(outdir, f"vimp{rank}.npy"), imp.cpu().numpy())
    with open(os.path.join(outdir, f"vrows{rank}.pkl"), "wb") as f:
        pickle.dump(_canon_rows(eng), f)
    eng.close()
    dist.destroy_process_group()


def test_two_rank_every_table_with_long_values(tmp_path):
    """testsblob (BLOB pk) and wide (composite pk) of corro-tests/src/lib.rs:32-52, TEXT / BLOB
    values longer than 16 bytes: the exchange routes interned rows by their canonical pk bytes,
    ships the bytes, re-keys them on the owner; the union of the two ranks' states equals one engine's
    merge of the whole batch, and every sender gets its changes' impacts back in its order."""
    import pickle
    import corrosion_amd as ca
    from tests.test_gpu_pk import INTERNED, SCHEMA, _changes
    world = 2
    mp.spawn(_var_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    got = []
    for r in range(world):
        with open(tmp_path / f"vrows{r}.pkl", "rb") as f:
            got += pickle.load(f)
    e = ca.MergeEngine(SCHEMA, capacity_hint=NV, interned=INTERNED)
    e.register_sites(synth.site_ids(6, 3))
    rows = _changes(np.random.default_rng(SEEDV), NV, 6)
    want_imp = e.apply(_pk_batch(e, rows), impact=True)
    want = _canon_rows(e)
    assert any(isinstance(t[5], bytes) for t in want) and any(isinstance(t[1], bytes) for t in want)
    assert sorted(got, key=repr) == want
    got_imp = np.concatenate([np.load(tmp_path / f"vimp{r}.npy") for r in range(world)])
    assert np.array_equal(got_imp, want_imp)


def test_partition_var_routes_unregistered_table_ids():
    """A change naming a table id past the schema goes through the every-table partition without
    touching the pk directory: routed like an INTEGER pk (rank_of), its record shipped unchanged, and
    refused by the owner's merge (cr-sqlite: no such table). Engines with interned tables and with
    none are both covered."""
    import torch
    import corrosion_amd as ca
    from corrosion_amd.dist import rank_of_np
    from tests.test_gpu_pk import INTERNED, SCHEMA
    for schema, interned in ((SCHEMA, INTERNED), ({"t": ["a"]}, ())):
        eng = ca.MergeEngine(schema, capacity_hint=1024, device=0, interned=interned)
        eng.register_sites(synth.site_ids(4, 3))
        n = 512
        bad_table = len(schema) + 7
        b = {"pk": np.arange(n, dtype=np.uint64) * 977,
             "table_cid": np.full(n, (bad_table << 16) | 1, np.uint32),
             "col_version": np.ones(n, np.int64), "db_version": np.ones(n, np.int64),
             "site": np.zeros(n, np.uint32), "cl": np.ones(n, np.uint32), "seq": np.zeros(n, np.uint32),
             "val0": np.arange(n, dtype=np.uint64)}
        dev = _to_dev(b)
        recs, var, counts, vcounts, perm = eng.partition_var(dev, 3, with_perm=True)
        torch.cuda.synchronize()
        want = np.bincount(rank_of_np(b["table_cid"], b["pk"], 3), minlength=3)
        assert counts == [int(c) for c in want] and vcounts == [0, 0, 0]
        got = eng.unpack_var(recs, var, counts, vcounts)
        assert np.array_equal(np.sort(got["pk"].cpu().numpy().view(np.uint64)), np.sort(b["pk"]))
        with pytest.raises(ca.CorroError):
            eng.apply(got)
        eng.close()


# ---- stream-ordered slot exchange (distributed_apply_slots) -------------------------------------
NS = 50000


def _slots_worker(rank, world, port, outdir, cap_scale, impact=False, chunk=0):
    import torch.distributed as dist
    import corrosion_amd as ca
    from corrosion_amd.dist import distributed_apply_slots, rank_of_np, slot_cap
    if chunk:  # (the received slots applied as several index-range chunks)
        os.environ["CORRO_HIP_CHUNK"] = str(chunk)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    full = synth.uniform_batch(NS, 16, 4000, 4, 77)
    lo, hi = rank * NS // world, (rank + 1) * NS // world
    eng = ca.MergeEngine({"t": ["a", "b", "c", "d"]}, capacity_hint=NS, device=0)
    eng.register_sites(synth.site_ids(16, 5))
    cap = max(1, int(slot_cap(hi - lo, world) * cap_scale))
    res = distributed_apply_slots(eng, _to_dev({k: v[lo:hi] for k, v in full.items()}), cap, impact=impact)
    nover = res[0] if impact else res
    if impact:
        np.save(os.path.join(outdir, f"simp{rank}.npy"), res[1].cpu().numpy())
    rows = eng.export()
    assert (rank_of_np(rows["table_cid"], rows["pk"], world) == rank).all()
    np.save(os.path.join(outdir, f"srows{rank}.npy"), np.array(rows_to_tuples(rows, with_ts=True), dtype=object),
            allow_pickle=True)
    np.save(os.path.join(outdir, f"sover{rank}.npy"), np.array([nover]))
    np.save(os.path.join(outdir, f"sdbv{rank}.npy"), np.asarray(eng.db_versions()))
    eng.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("impact", [False, True], ids=["no_impacts", "impacts"])
@pytest.mark.parametrize("cap_scale,chunk", [(1.0, 0), (0.3, 0), (1.0, 4096)],
                         ids=["slots_fit", "slots_overflow_repeat", "slots_fit_chunked"])
def test_two_rank_slot_exchange_equals_single_engine(tmp_path, cap_scale, chunk, impact):
    """distributed_apply_slots: fixed slots, equal-split all-to-alls on the engine's stream, the merge
    straight from the received slots (corro_apply_slots: no unpack pass, padding skipped); with slots
    too small (0.3 x) every rank overflows, merges nothing in the slot pass and repeats with the
    exact-size exchange -- the union of the rank states equals one engine's merge of the whole batch
    either way. With impacts the flags come back to their senders on the stream (a third equal-split
    all-to-all + the partition's permutation) and equal the single engine's, in each rank's order.
    `chunked`: the receivers apply their slot layout in 4096-record index ranges (a batch larger than
    one apply chunk), whose boundaries fall inside the slots."""
    import corrosion_amd as ca
    world = 2
    mp.spawn(_slots_worker, args=(world, _free_port(), str(tmp_path), cap_scale, impact, chunk), nprocs=world,
             join=True)
    got = []
    for r in range(world):
        got += [tuple(x) for x in np.load(tmp_path / f"srows{r}.npy", allow_pickle=True)]
    nover = int(np.load(tmp_path / "sover0.npy")[0])
    assert (nover == 0) == (cap_scale == 1.0)
    from oracle import oracle as O
    e = ca.MergeEngine({"t": ["a", "b", "c", "d"]}, capacity_hint=NS)
    e.register_sites(synth.site_ids(16, 5))
    batch = synth.uniform_batch(NS, 16, 4000, 4, 77)
    want_imp = e.apply(batch, impact=True)
    assert sorted(got) == rows_to_tuples(e.export(), with_ts=True)
    if impact:
        got_imp = np.concatenate([np.load(tmp_path / f"simp{r}.npy") for r in range(world)])
        assert np.array_equal(got_imp, want_imp)
    dbv = np.max([np.load(tmp_path / f"sdbv{r}.npy") for r in range(world)], axis=0)
    assert list(dbv) == list(e.db_versions())
    f = O.Fold(synth.site_ids(16, 5))  # (the single engine, so the ranks' union, against the oracle)
    f.apply(batch)
    assert O.rows_diff(e.export(), f.export()) is None
    assert list(e.db_versions()) == list(f.db_versions())


@pytest.mark.gpu
@pytest.mark.parametrize("bad", ["site", "table", "col_version", None])
def test_slot_partition_validates_and_marks_counts(bad):
    """corro_partition_slots validates what it packs (the apply's pre-write checks) and marks every
    destination's count (bit 63) when the batch fails them: the receiver then sees an overflowed slot
    and applies nothing -- even when its slots span several apply chunks, whose whole-layout validation
    pass it no longer runs -- and the exchange repeats through the validating apply. A valid batch is
    unmarked and merges as one engine would."""
    import torch
    import corrosion_amd as ca
    from corrosion_amd.dist import slot_cap
    full = synth.uniform_batch(NS, 16, 4000, 4, 77)
    if bad == "site":
        full["site"][NS // 3] = 999
    elif bad == "table":
        full["table_cid"][NS // 2] = (7 << 16) | 1
    elif bad == "col_version":
        full["cl"][NS // 4] = 2
        full["col_version"][NS // 4] = -5
    dev = _to_dev(full)
    world = 2
    cap = slot_cap(NS, world)
    eng = ca.MergeEngine({"t": ["a", "b", "c", "d"]}, capacity_hint=NS, device=0)
    eng.register_sites(synth.site_ids(16, 5))
    recs, cnt = eng.partition_slots(dev, world, cap)
    torch.cuda.synchronize()
    marked = (cnt.cpu() < 0).tolist()  # (bit 63 reads as a negative int64)
    assert all(marked) == (bad is not None) and any(marked) == (bad is not None)
    os.environ["CORRO_HIP_CHUNK"] = "4096"  # (the slot layout as several chunks)
    try:
        _, over = eng.apply_slots(recs, world, cap, cnt)
    finally:
        del os.environ["CORRO_HIP_CHUNK"]
    torch.cuda.synchronize()
    assert int(over.item()) == (1 if bad else 0)
    if bad:
        assert eng.count() == 0
        with pytest.raises(ca.CorroError):
            eng.apply(dev)
    else:
        e = ca.MergeEngine({"t": ["a", "b", "c", "d"]}, capacity_hint=NS)
        e.register_sites(synth.site_ids(16, 5))
        e.apply(full)
        assert rows_to_tuples(eng.export(), with_ts=True) == rows_to_tuples(e.export(), with_ts=True)


# ---- the multi-rank path at scale, against the oracle ---------------------------------------------
# (the tests above pin the exchange at 6,000-50,000 changes; here a config-5-shaped adversarial batch
# of 4M changes -- Zipf-hot rows, so every rank's merge runs the device-wide overflow fold -- and a
# config-2-shaped INTEGER batch of 2^24 changes through the stream-ordered slot path, with impacts,
# each against the oracle's pk-sharded fold of the whole batch: every impact flag in each sender's
# order, the union of the rank states by the order-independent digest of every output field (a
# mismatch prints the row-by-row report), crsql_db_versions)
NL_ADV, NL_INT, NL_CHUNKED = 4_000_000, 1 << 24, 1 << 26
CHUNK_FORCED = 1 << 23


def _large_worker(rank, world, port, outdir, kind):
    import torch
    import torch.distributed as dist
    import corrosion_amd as ca
    from corrosion_amd.dist import distributed_apply, distributed_apply_slots, rank_of_np, slot_cap
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    if kind == "integer_slots_chunked":  # (each receiver applies its slot layout in index-range chunks)
        os.environ["CORRO_HIP_CHUNK"] = str(CHUNK_FORCED)
    if kind == "adversarial":
        n, seed = NL_ADV, synth.config_seed(5)
        schema, sites = synth.adversarial_schema(8), synth.site_ids(1000, seed)
        full = synth.adversarial_batch(n, 1000, 8, 1 << 20, seed)
    else:
        n, seed = (NL_CHUNKED if kind == "integer_slots_chunked" else NL_INT), synth.config_seed(2)
        schema, sites = {"t": ["a", "b", "c", "d"]}, synth.site_ids(1000, 1)
        full = synth.uniform_batch(n, 1000, 1 << 22, 4, seed)
    lo, hi = rank * n // world, (rank + 1) * n // world
    eng = ca.MergeEngine(schema, capacity_hint=n // world, device=0)
    eng.register_sites(sites)
    part = _to_dev({k: v[lo:hi] for k, v in full.items()})
    del full
    if kind == "adversarial":
        imp = distributed_apply(eng, part, impact=True)
        assert eng.metrics()["overflow_rounds"] >= 1  # the hot-row regime on this rank
    else:
        cap = slot_cap(hi - lo, world)
        nover, imp = distributed_apply_slots(eng, part, cap, impact=True)
        assert nover == 0
        np.save(os.path.join(outdir, f"lchunks{rank}.npy"), np.array(-(-(world * cap) // CHUNK_FORCED)))
    torch.cuda.synchronize()
    np.save(os.path.join(outdir, f"limp{rank}.npy"), imp.cpu().numpy())
    rows = eng.export()
    assert (rank_of_np(rows["table_cid"], rows["pk"], world) == rank).all()
    assert not rows.get("long_values")  # (values of at most 16 bytes: the rows are plain arrays)
    np.savez(os.path.join(outdir, f"lrows{rank}.npz"), **{k: v for k, v in rows.items() if k != "long_values"})
    np.save(os.path.join(outdir, f"ldbv{rank}.npy"), np.asarray(eng.db_versions()))
    eng.close()
    dist.destroy_process_group()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("kind", ["adversarial", "integer_slots"])
def test_two_rank_large_batch_vs_sharded_oracle(tmp_path, kind):
    from oracle import oracle as O
    world = 2
    mp.spawn(_large_worker, args=(world, _free_port(), str(tmp_path), kind), nprocs=world, join=True)
    if kind == "adversarial":
        n, seed = NL_ADV, synth.config_seed(5)
        sites, batch = synth.site_ids(1000, seed), synth.adversarial_batch(NL_ADV, 1000, 8, 1 << 20, seed)
    else:
        n, seed = NL_INT, synth.config_seed(2)
        sites, batch = synth.site_ids(1000, 1), synth.uniform_batch(NL_INT, 1000, 1 << 22, 4, seed)
    fold = O.ShardedFold(sites, nshards=64, nthreads=16)
    want_imp = fold.apply(batch, impact=True)
    got_imp = np.concatenate([np.load(tmp_path / f"limp{r}.npy") for r in range(world)])
    assert np.array_equal(got_imp, want_imp), "impact flags differ from the oracle"
    parts = [dict(np.load(tmp_path / f"lrows{r}.npz")) for r in range(world)]
    rows = {k: np.concatenate([p[k] for p in parts]) for k in parts[0]}
    if O.rows_digest(rows) != fold.digest():
        pytest.fail(f"{kind}: the ranks' union differs from the oracle:\n" + str(O.rows_diff(rows, fold.export())))
    dbv = np.max([np.load(tmp_path / f"ldbv{r}.npy") for r in range(world)], axis=0)
    assert np.array_equal(dbv, fold.db_versions())
    print(f"{kind}: {n} changes over {world} ranks, {len(rows['pk'])} clock rows bit-exact")


# ---- failure on one rank fails the call on every rank ----------------
def _fail_worker(rank, world, port, outdir, case):
    import datetime
    import torch.distributed as dist
    import corrosion_amd as ca
    from corrosion_amd.dist import distributed_apply, distributed_apply_slots, slot_cap
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=60))
    full = synth.uniform_batch(NS, 16, 4000, 4, 77)
    lo, hi = rank * NS // world, (rank + 1) * NS // world
    mine = {k: v[lo:hi].copy() for k, v in full.items()}
    if case.startswith("invalid") and rank == 0:
        mine["site"][len(mine["site"]) // 2] = 999  # (an unregistered site ordinal: the receiver refuses it)
    eng = ca.MergeEngine({"t": ["a", "b", "c", "d"]}, capacity_hint=NS, device=0)
    eng.register_sites(synth.site_ids(16, 5))
    if case == "apply_slots_rank1" and rank == 1:
        os.environ["CORRO_FAULT"] = "apply_slots"
    if case == "partition_slots_rank0" and rank == 0:
        os.environ["CORRO_FAULT"] = "partition_slots"
    try:
        if case == "invalid_exact":
            distributed_apply(eng, _to_dev(mine), impact=True)
        else:
            distributed_apply_slots(eng, _to_dev(mine), slot_cap(hi - lo, world), impact=True)
        out = "ok"
    except ca.CorroError as e:
        out = "raised: " + str(e)
    except RuntimeError as e:
        out = "hung: " + str(e)
    os.environ.pop("CORRO_FAULT", None)
    open(os.path.join(outdir, f"f{rank}.txt"), "w").write(out)
    eng.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("case", ["apply_slots_rank1", "partition_slots_rank0", "invalid_slots", "invalid_exact"])
def test_one_rank_failure_raises_on_every_rank(tmp_path, case):
    """A rank-local failure inside the multi-rank step (an injected CORRO_FAULT in the slot merge or
    the slot partition, or an invalid change: the sender's validation marks its slots, the receivers
    repeat through the exact-size exchange whose merge refuses it -- with impact flags, whose
    collectives follow that merge) makes every rank raise CorroError; none blocks in a collective."""
    world = 2
    mp.spawn(_fail_worker, args=(world, _free_port(), str(tmp_path), case), nprocs=world, join=True)
    got = [open(tmp_path / f"f{r}.txt").read() for r in range(world)]
    assert all(g.startswith("raised") for g in got), got


def test_unpack_var_refuses_bytes_outside_the_received_buffer():
    """corro_unpack_var checks each record's shipped pk / value span against the received
    bytes (and a pk length against the 24-bit reference) on the device: a corrupt record is
    CORRO_E_INVALID, never a read past the buffer."""
    import torch
    import corrosion_amd as ca
    from tests.test_gpu_pk import INTERNED, SCHEMA, _changes
    rows = _changes(np.random.default_rng(4), 400, 4)
    eng = ca.MergeEngine(SCHEMA, capacity_hint=4096, device=0, interned=INTERNED)
    eng.register_sites(synth.site_ids(6, 3))
    dev = {}
    for k, v in _pk_batch(eng, rows).items():
        v = np.ascontiguousarray(v)
        dev[k] = torch.from_numpy(v.view(np.int64) if v.dtype == np.uint64 else
                                  (v.view(np.int32) if v.dtype == np.uint32 else v)).cuda()
    recs, var, counts, vcounts, _ = eng.partition_var(dev, 1)
    assert vcounts[0] > 0
    eng.unpack_var(recs.clone(), var, counts, vcounts)  # (intact: accepted)
    r = recs.cpu().numpy().view(np.uint32).reshape(-1, 20)
    j = int(np.nonzero(r[:, 18])[0][0])  # a record shipping pk bytes (pad[1] = its pk length)
    for word, val in ((17, 1 << 30), (18, 1 << 24), (19, 1 << 28)):  # pad[0] offset, pad[1] pk length, pad[2] value size
        bad = r.copy()
        bad[j, word] = val
        with pytest.raises(ca.CorroError):
            eng.unpack_var(torch.from_numpy(bad.view(np.uint8).reshape(-1)).cuda(), var, counts, vcounts)
    eng.close()


@pytest.mark.timeout(900)
def test_two_rank_chunked_slot_receiver_vs_sharded_oracle(tmp_path):
    """the chunked slot receiver config 3 runs at full size, pinned to the oracle at
    2^26 global changes -- each receiver's ~2^25 slot records applied as index-range chunks of 2^23
    (CORRO_HIP_CHUNK; >= 4 chunks, each merging into the state the earlier ones wrote), with impacts,
    against the oracle's pk-sharded fold: every flag in each sender's order, the ranks' union row by
    row, db_versions."""
    from oracle import oracle as O
    world = 2
    mp.spawn(_large_worker, args=(world, _free_port(), str(tmp_path), "integer_slots_chunked"), nprocs=world,
             join=True)
    n = NL_CHUNKED
    sites, batch = synth.site_ids(1000, 1), synth.uniform_batch(n, 1000, 1 << 22, 4, synth.config_seed(2))
    fold = O.ShardedFold(sites, nshards=64, nthreads=16)
    want_imp = fold.apply(batch, impact=True)
    del batch
    got_imp = np.concatenate([np.load(tmp_path / f"limp{r}.npy") for r in range(world)])
    assert np.array_equal(got_imp, want_imp), "impact flags differ from the oracle"
    parts = [dict(np.load(tmp_path / f"lrows{r}.npz")) for r in range(world)]
    rows = {k: np.concatenate([p[k] for p in parts]) for k in parts[0]}
    chunks = [int(np.load(tmp_path / f"lchunks{r}.npy")) for r in range(world)]
    assert min(chunks) >= 4, chunks
    diff = O.rows_diff(rows, fold.export())
    assert diff is None, str(diff)
    dbv = np.max([np.load(tmp_path / f"ldbv{r}.npy") for r in range(world)], axis=0)
    assert np.array_equal(dbv, fold.db_versions())
