"""Two ranks on one GPU box: device pk-hash partition (HIP) + all-to-all exchange (gloo through host
memory here; RCCL on a multi-GPU node) + per-rank device merge. The union of the rank states must
equal the single-engine merge of the whole batch, bit for bit."""
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
    e = ca.MergeEngine(synth.adversarial_schema(NT), capacity_hint=N)
    e.register_sites(synth.site_ids(8, SEED))
    want_imp = e.apply(synth.adversarial_batch(N, 8, NT, 500, SEED), impact=True)
    assert sorted(got) == rows_to_tuples(e.export(), with_ts=True)
    # per-change impacts come back to each sender in its own order (reverse all-to-all + permutation)
    got_imp = np.concatenate([np.load(tmp_path / f"imp{r}.npy") for r in range(world)])
    assert np.array_equal(got_imp, want_imp)


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
