"""Full-size parity (the north-star criterion and BASELINE's stated sizes), in the GPU suite:

  * config 3: 2^29 = 536,870,912 column changes (pk space 2^25, 1000 actors, 4 INTEGER columns,
    cl = 1), merged on one MI355X as ONE batch, and as 8 consecutive 2^26 batches folded into one
    state (each batch into the state the previous ones left: the in-place row store), checked against
    the oracle's pk-sharded fold (oracle/crsql_fold.c of_apply_sharded, the sequential rules run per
    shard on the host cores): every impact flag, the crsql_changes rows through an order-independent
    digest of every output field (row count, sum and xor of per-row 64-bit hashes; a mismatch prints
    the row-by-row report of oracle.rows_diff), crsql_db_versions;
  * config 5: the adversarial mix at its stated 64M size (8 tables, Zipf(1.1) hot pks over 2^20 per
    table, 30 % sentinel deletes / resurrects, mixed INTEGER / REAL / TEXT / BLOB / NULL values), two
    64M batches folded into one state with impact flags -- the regime where ~57M records per apply
    take the device-wide overflow fold with the row store's prior-row lookups -- against the same
    pk-sharded oracle fold, every output row compared field by field (oracle.rows_diff) and by digest;
  * config 4: 1M node pairs x 64 sparse actors from a 100k-actor universe (64M need-diff entries),
    the device need diff against the oracle restatement (oracle/ranges.c, threaded over entry
    chunks), every output array equal.
The oracle is the checker only."""
import time

import numpy as np
import pytest

import synth
from oracle import oracle as O

pytestmark = pytest.mark.gpu

N3, PK3, ACT = 1 << 29, 1 << 25, 1000


def _host(b):
    hb = {k: v.cpu().numpy() for k, v in b.items()}
    for k in ("table_cid", "cl", "seq", "site"):
        hb[k] = hb[k].view(np.uint32)
    for k in ("pk", "val0"):
        hb[k] = hb[k].view(np.uint64)
    return hb


def _config3(batches):
    import torch
    import corrosion_amd as ca
    sites = synth.site_ids(ACT, 1)
    eng = ca.MergeEngine({"t": ["a", "b", "c", "d"]}, capacity_hint=N3 // batches, device=0)
    eng.register_sites(sites)
    fold = O.ShardedFold(sites, nshards=64, nthreads=16)
    per = N3 // batches
    t_gpu = []
    for k in range(batches):
        b = synth.uniform_batch_torch(per, ACT, PK3, 4, seed=synth.config_seed(3) + k, device="cuda")
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        imp = eng.apply(b, impact=True)
        torch.cuda.synchronize()
        t_gpu.append(time.perf_counter() - t0)
        imp = imp.cpu().numpy()
        hb = _host(b)
        del b
        torch.cuda.empty_cache()
        ref = fold.apply(hb)
        assert np.array_equal(imp, ref), f"batch {k}: impact flags differ"
        del hb, imp, ref
    rows = eng.export()
    dg = O.rows_digest(rows)
    if dg != fold.digest():  # (where: the row-by-row report)
        pytest.fail("config 3 state differs from the oracle:\n" + str(O.rows_diff(rows, fold.export())))
    del rows
    assert np.array_equal(eng.db_versions(), fold.db_versions())
    print(f"config 3, {batches} batch(es): {dg[0]} clock rows bit-exact; GPU apply s per batch "
          + ", ".join(f"{t:.3f}" for t in t_gpu))
    eng.close()


def test_config3_512m_one_batch_vs_sharded_oracle():
    _config3(1)


def test_config3_512m_eight_batch_fold_vs_sharded_oracle():
    _config3(8)


def _dev(b):
    import torch
    return {k: torch.from_numpy(v.view(np.int64) if v.dtype == np.uint64 else
                                (v.view(np.int32) if v.dtype == np.uint32 else v)).cuda() for k, v in b.items()}


@pytest.mark.timeout(1200)
@pytest.mark.parametrize("impact", [True, False], ids=["impacts", "no_impacts"])
def test_config5_64m_two_batch_fold_vs_sharded_oracle(impact):
    """With impacts every change keeps its place in the fold; without them the overflow fold reduces
    hot rows to their last epoch's changes first (ovf_kernels.h) -- both against the same oracle."""
    import torch
    import corrosion_amd as ca
    n = 64_000_000
    seed = synth.config_seed(5)
    sites = synth.site_ids(1000, seed)
    eng = ca.MergeEngine(synth.adversarial_schema(8), capacity_hint=n, device=0)
    eng.register_sites(sites)
    fold = O.ShardedFold(sites, nshards=64, nthreads=16)
    import time
    t0 = time.time()
    for k in range(2):
        b = synth.adversarial_batch(n, 1000, 8, 1 << 20, seed + k)
        print(f"batch {k} generated at {time.time() - t0:.0f} s", flush=True)
        d = _dev(b)
        imp = eng.apply(d, impact=impact)
        imp = imp.cpu().numpy() if impact else None
        print(f"batch {k} applied on the GPU at {time.time() - t0:.0f} s", flush=True)
        del d
        torch.cuda.empty_cache()
        ref = fold.apply(b, impact=impact)
        print(f"batch {k} folded by the oracle at {time.time() - t0:.0f} s", flush=True)
        if impact:
            assert np.array_equal(imp, ref), f"config 5 batch {k}: impact flags differ"
        del b, imp, ref
    m = eng.metrics()
    assert m["overflow_rounds"] >= 2          # the hot-row regime was exercised
    rows = eng.export()
    dg = O.rows_digest(rows)
    # every row compared field by field against the oracle's rows (8 M rows), and the digest too
    rep = O.rows_diff(rows, fold.export())
    assert rep is None, "config 5 state differs from the oracle:\n" + rep
    del rows
    assert dg == fold.digest()
    assert np.array_equal(eng.db_versions(), fold.db_versions())
    print(f"config 5, 2 x 64M folded: {dg[0]} clock rows bit-exact, row by row")
    eng.close()


def test_config4_full_size_vs_oracle():
    import torch
    import corrosion_amd as ca
    from corrosion_amd.sync import _needs_device
    ent = synth.sync_entries_torch(1_000_000, 64, synth.config_seed(4), device="cuda")
    e = ca.MergeEngine({"t": ["a"]}, capacity_hint=1024)
    got = _needs_device(e, ent)
    host = {k: v.cpu().numpy() for k, v in ent.items()}
    del ent
    torch.cuda.empty_cache()
    exp = O.needs_parallel(host, nthreads=16)
    assert len(host["their_head"]) == 64_000_000
    for k in ("need_off", "seq_off", "kind", "start", "end", "sr_off", "sr_n", "s_start", "s_end"):
        g = got[k].cpu().numpy() if hasattr(got[k], "cpu") else got[k]
        assert np.array_equal(g.view(exp[k].dtype) if g.dtype != exp[k].dtype and g.itemsize == exp[k].itemsize
                              else g, exp[k]), k
    e.close()


def test_config4_full_size_packed_equals_two_pass():
    """Config 4 at its stated size (1M node pairs x 64 actors = 64M entries): the packed one-pass
    kernel's needs equal the two-pass kernel's (itself checked against the oracle above), compared
    on the device slot by slot."""
    import torch
    import corrosion_amd as ca
    from corrosion_amd.sync import _needs_device, _needs_device_packed
    ent = synth.sync_entries_torch(1_000_000, 64, synth.config_seed(4), device="cuda")
    e = ca.MergeEngine({"t": ["a"]}, capacity_hint=1024)
    a = _needs_device(e, ent)
    b = _needs_device_packed(e, ent)
    del ent
    cnt = b["need_count"].to(torch.int64)
    assert bool((cnt == a["need_off"][1:] - a["need_off"][:-1]).all())
    T = int(a["need_off"][-1])
    slot = torch.repeat_interleave(b["need_off"] - a["need_off"][:-1], cnt) + torch.arange(T, device="cuda")
    rng = b["range"].view(-1, 2)
    kind = b["kind"][slot]
    assert bool((kind == a["kind"]).all())
    lo, hi = rng[slot, 0], rng[slot, 1]
    part = kind == 1
    assert bool((lo == a["start"]).all())
    assert bool((torch.where(part, lo, hi) == a["end"]).all())
    assert bool((torch.where(part, hi & 0xFFFFFF, 0) == a["sr_n"]).all())
    first = torch.where(part, hi >> 24, 0)
    sr = a["sr_n"]
    Ts = int(sr.sum())
    assert Ts == int(a["seq_off"][-1])
    src = torch.repeat_interleave(first, sr) + (torch.arange(Ts, device="cuda")
                                               - torch.repeat_interleave(a["sr_off"], sr))
    assert bool((b["s_start"][src] == a["s_start"]).all()) and bool((b["s_end"][src] == a["s_end"]).all())
    e.close()
