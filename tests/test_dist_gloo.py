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
