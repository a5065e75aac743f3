"""World-size-2 rehearsal of the multi-GPU path on CPU (gloo): rows sharded by owner rank,
exchanged with all-to-all-v, merged per rank. The sharded result must equal the single-node
merge of the whole batch. The per-rank merge here is the CPU oracle (the checker); the product
partition kernel is checked against rank_of_np on the GPU (tests/test_gpu_merge.py)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import synth
from corrosion_amd.dist import rank_of_np
from tests._util import rows_to_tuples

N, SEED = 6000, 91


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, outdir):
    import torch
    import torch.distributed as dist
    from corrosion_amd.dist import exchange
    from oracle import oracle as O
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sites = synth.site_ids(8, SEED)
    full = synth.adversarial_batch(N, 8, 2, 300, SEED)
    lo, hi = rank * N // world, (rank + 1) * N // world
    mine = {k: v[lo:hi] for k, v in full.items()}
    dest = rank_of_np(mine["table_cid"], mine["pk"], world)
    order = np.argsort(dest, kind="stable")
    counts = np.bincount(dest, minlength=world).tolist()
    parts = {k: torch.from_numpy(np.ascontiguousarray(v[order]).view(
        np.int64 if v.dtype == np.uint64 else (np.int32 if v.dtype == np.uint32 else v.dtype))) for k, v in mine.items()}
    got = exchange(parts, counts)
    recv = {k: got[k].numpy().view(full[k].dtype) for k in full}
    assert (rank_of_np(recv["table_cid"], recv["pk"], world) == rank).all()
    f = O.Fold(sites)
    f.apply(recv)
    np.save(os.path.join(outdir, f"rows{rank}.npy"), np.array(rows_to_tuples(f.export(), with_ts=True), dtype=object),
            allow_pickle=True)
    dist.destroy_process_group()


def test_sharded_merge_equals_single_node(tmp_path):
    from oracle import oracle as O
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    got = []
    for r in range(world):
        got += [tuple(x) for x in np.load(tmp_path / f"rows{r}.npy", allow_pickle=True)]
    f = O.Fold(synth.site_ids(8, SEED))
    f.apply(synth.adversarial_batch(N, 8, 2, 300, SEED))
    assert sorted(got) == rows_to_tuples(f.export(), with_ts=True)


REC48 = np.dtype([("pk", "<u8"), ("cv", "<i8"), ("dbv", "<i8"), ("v0", "<u8"), ("tcid", "<u4"), ("cl", "<u4"),
                  ("seq", "<u4"), ("site", "<u4")])


def _rec_worker(rank, world, port, outdir):
    """corro_partition_packed's record layout, packed on the host: one all-to-all of whole 48-B
    records moves every field, in source-rank order."""
    import torch
    import torch.distributed as dist
    from corrosion_amd.dist import exchange_records
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    full = synth.uniform_batch(N, 8, 300, 4, SEED)
    lo, hi = rank * N // world, (rank + 1) * N // world
    mine = {k: v[lo:hi] for k, v in full.items()}
    dest = rank_of_np(mine["table_cid"], mine["pk"], world)
    order = np.argsort(dest, kind="stable")
    recs = np.zeros(hi - lo, REC48)
    for f, k in (("pk", "pk"), ("cv", "col_version"), ("dbv", "db_version"), ("v0", "val0"), ("tcid", "table_cid"),
                 ("cl", "cl"), ("seq", "seq"), ("site", "site")):
        recs[f] = mine[k][order]
    counts = np.bincount(dest, minlength=world).tolist()
    got, rcounts = exchange_records(torch.from_numpy(recs.view(np.uint8).copy()), 48, counts)
    r = got.numpy().view(REC48)
    assert len(r) == sum(rcounts)
    assert (rank_of_np(r["tcid"], r["pk"], world) == rank).all()
    np.save(os.path.join(outdir, f"recs{rank}.npy"), r)
    dist.destroy_process_group()


def test_packed_record_exchange_preserves_order(tmp_path):
    world = 2
    mp.spawn(_rec_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    full = synth.uniform_batch(N, 8, 300, 4, SEED)
    dest = rank_of_np(full["table_cid"], full["pk"], world)
    for r in range(world):
        got = np.load(tmp_path / f"recs{r}.npy")
        want = np.nonzero(dest == r)[0]  # rank-major global order = application order
        assert np.array_equal(got["pk"], full["pk"][want])
        assert np.array_equal(got["seq"], full["seq"][want])
        assert np.array_equal(got["dbv"], full["db_version"][want])
