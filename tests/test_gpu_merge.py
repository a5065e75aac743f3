"""GPU parity of the batched merge (libcorro_hip.so through the C ABI) against the CPU oracle
restatement of cr-sqlite's crsql_changes INSERT (oracle/crsql_fold.c) and the golden KATs.
Bar: bit-exact crsql_changes rows, impacts and crsql_db_versions."""
import numpy as np
import pytest

import synth
from oracle import oracle as O
from tests._util import batch_from_changes, expected_rows, load_golden, rows_to_tuples, site_table

pytestmark = pytest.mark.gpu

SCHEMA_T = {"t": ["a", "b", "c"]}
MERGE = load_golden("merge_kats.json")


def engine(schema, cap=1 << 16, sites=None):
    import corrosion_amd as ca
    e = ca.MergeEngine(schema, capacity_hint=cap)
    e.register_sites(site_table() if sites is None else sites)
    return e


def compare(eng, fold, with_ts=False):
    got = rows_to_tuples(eng.export(), with_ts=with_ts)
    exp = rows_to_tuples(fold.export(), with_ts=with_ts)
    assert len(got) == len(exp)
    assert got == exp
    nd = fold.nsites
    assert list(eng.db_versions()[:nd]) == list(fold.db_versions())


@pytest.mark.parametrize("case", MERGE["cases"], ids=[c["name"][:3] for c in MERGE["cases"]])
def test_kats_gpu(case):
    e = engine(SCHEMA_T)
    imp = e.apply(batch_from_changes(case["changes"]), impact=True)
    got = [t[:11] for t in rows_to_tuples(e.export())]
    assert got == expected_rows(case["rows"])
    assert list(np.cumsum(imp)) == case["impacted"]


@pytest.mark.parametrize("case", MERGE["cases"], ids=[c["name"][:3] for c in MERGE["cases"]])
def test_kats_gpu_one_change_per_batch(case):
    """Folding batch-by-batch equals one batch (state is the prefix of application order)."""
    e = engine(SCHEMA_T)
    b = batch_from_changes(case["changes"])
    for i in range(len(b["pk"])):
        e.apply({k: v[i:i + 1] for k, v in b.items()})
    assert [t[:11] for t in rows_to_tuples(e.export())] == expected_rows(case["rows"])


def test_kats_gpu_no_impact_path():
    """Without impact output the fast/general split is used; results identical."""
    for case in MERGE["cases"]:
        e = engine(SCHEMA_T)
        e.apply(batch_from_changes(case["changes"]))
        assert [t[:11] for t in rows_to_tuples(e.export())] == expected_rows(case["rows"]), case["name"]


def test_db_versions_gpu():
    c = MERGE["db_versions_case"]
    e = engine(SCHEMA_T)
    e.apply(batch_from_changes(c["changes"]))
    dv = e.db_versions()
    for site, v in c["db_versions"].items():
        assert dv[int(site)] == v
    assert dv[0] == -1


@pytest.mark.parametrize("n,npk,seed", [(1000, 50, 1), (20000, 3000, 2), (200000, 40000, 3)])
def test_uniform_cl1_vs_oracle(n, npk, seed):
    sites = synth.site_ids(16, seed)
    b = synth.uniform_batch(n, 16, npk, 4, seed)
    e = engine({"t": ["a", "b", "c", "d"]}, cap=n, sites=sites)
    f = O.Fold(sites)
    e.apply(b)
    f.apply(b)
    compare(e, f)


@pytest.mark.parametrize("malformed", [False, True])
@pytest.mark.parametrize("seed", [11, 12, 13])
def test_adversarial_vs_oracle(seed, malformed):
    sites = synth.site_ids(8, seed)
    b = synth.adversarial_batch(30000, 8, 3, 400, seed, malformed=malformed)
    e = engine(synth.adversarial_schema(3), cap=30000, sites=sites)
    f = O.Fold(sites)
    imp_e = e.apply(b, impact=True)
    imp_f = f.apply(b)
    compare(e, f, with_ts=True)
    assert np.array_equal(imp_e, imp_f)


def test_adversarial_multi_batch_fold():
    """Several batches in sequence (prior state as prefix), with and without impact output."""
    seed = 21
    sites = synth.site_ids(8, seed)
    e = engine(synth.adversarial_schema(2), cap=20000, sites=sites)
    f = O.Fold(sites)
    for k in range(6):
        b = synth.adversarial_batch(5000, 8, 2, 300, seed + k)
        if k % 2:
            assert np.array_equal(e.apply(b, impact=True), f.apply(b))
        else:
            e.apply(b)
            f.apply(b)
        compare(e, f, with_ts=True)


def test_mixed_cl1_then_adversarial():
    """Fast-path state (cl=1 rows) then deletes/resurrects on the same rows."""
    seed = 31
    sites = synth.site_ids(8, seed)
    e = engine(synth.adversarial_schema(1), cap=50000, sites=sites)
    f = O.Fold(sites)
    b1 = synth.uniform_batch(40000, 8, 2000, 4, seed)
    b1["table_cid"] = (b1["table_cid"] & 0xFFFF).astype(np.uint32)
    e.apply(b1)
    f.apply(b1)
    compare(e, f)
    b2 = synth.adversarial_batch(20000, 8, 1, 2000, seed + 1, zipf=0, wide=False)
    e.apply(b2)
    f.apply(b2)
    compare(e, f, with_ts=False)


def test_hot_rows_overflow_buckets():
    """Zipf-hot rows make buckets larger than LDS: the global-scratch path must agree."""
    seed = 41
    sites = synth.site_ids(8, seed)
    b = synth.adversarial_batch(60000, 8, 1, 50, seed, zipf=1.1)
    e = engine(synth.adversarial_schema(1), cap=64, sites=sites)  # tiny bucket table
    f = O.Fold(sites)
    assert np.array_equal(e.apply(b, impact=True), f.apply(b))
    compare(e, f, with_ts=True)


def test_fast_path_overflow_cl1():
    seed = 42
    sites = synth.site_ids(4, seed)
    b = synth.uniform_batch(50000, 4, 20000, 3, seed)
    e = engine(SCHEMA_T, cap=64, sites=sites)
    f = O.Fold(sites)
    e.apply(b)
    f.apply(b)
    compare(e, f)


def test_device_resident_batch():
    import torch
    seed = 51
    sites = synth.site_ids(16, seed)
    b = synth.uniform_batch(100000, 16, 10000, 4, seed)
    dev = {k: torch.from_numpy(v.view(np.int64) if v.dtype == np.uint64 else
                               (v.view(np.int32) if v.dtype == np.uint32 else v)).cuda() for k, v in b.items()}
    e = engine({"t": ["a", "b", "c", "d"]}, cap=100000, sites=sites)
    f = O.Fold(sites)
    e.apply(dev)
    f.apply(b)
    compare(e, f)


def test_reset_and_reapply():
    seed = 61
    sites = synth.site_ids(4, seed)
    b = synth.uniform_batch(10000, 4, 1000, 3, seed)
    e = engine(SCHEMA_T, cap=10000, sites=sites)
    e.apply(b)
    first = rows_to_tuples(e.export())
    e.reset()
    assert e.count() == 0
    e.apply(b)
    assert rows_to_tuples(e.export()) == first


def test_errors_leave_state_untouched():
    import corrosion_amd as ca
    e = engine(SCHEMA_T)
    b = batch_from_changes([[1, {"t": "int", "v": 5}, 1, 7, 1, 1]])
    e.apply(b)
    before = rows_to_tuples(e.export())
    bad = batch_from_changes([[7, {"t": "int", "v": 5}, 2, 8, 1, 1]])  # cid 7 does not exist
    with pytest.raises(ca.CorroError) as ex:
        e.apply(bad)
    assert ex.value.code == -5
    assert rows_to_tuples(e.export()) == before
    bad = batch_from_changes([[1, {"t": "int", "v": 5}, 2, 8, 99, 1]])  # unknown site ordinal
    with pytest.raises(ca.CorroError):
        e.apply(bad)
    assert rows_to_tuples(e.export()) == before
    assert e.lookup("t", "b") == 2 and e.lookup("t", "-1") == 0
    with pytest.raises(ca.CorroError):
        e.lookup("t", "zz")


def test_exported_state_reapplied_reproduces_itself():
    """A state's clock rows, replayed as one batch on an empty engine, give the same rows
    (the state is a valid prefix of the application order; used to re-seed the engine)."""
    seed = 71
    sites = synth.site_ids(8, seed)
    e = engine(synth.adversarial_schema(2), cap=20000, sites=sites)
    for k in range(3):
        e.apply(synth.adversarial_batch(6000, 8, 2, 200, seed + k))
    rows = e.export()
    replay = {"pk": rows["pk"], "table_cid": rows["table_cid"], "col_version": rows["col_version"],
              "db_version": rows["db_version"], "cl": rows["cl"].astype(np.uint32), "seq": rows["seq"],
              "site": rows["site"], "val0": rows["val0"], "val1": rows["val1"],
              "val_type": rows["val_type"], "val_len": rows["val_len"], "ts": rows["ts"]}
    e2 = engine(synth.adversarial_schema(2), cap=20000, sites=sites)
    e2.apply(replay)
    assert rows_to_tuples(e2.export(), with_ts=True) == rows_to_tuples(rows, with_ts=True)


@pytest.mark.parametrize("nranks", [1, 2, 3, 8])
def test_partition_ranks_stable(nranks):
    """corro_partition_ranks == stable partition by rank_of (host mirror)."""
    import torch
    from corrosion_amd.dist import rank_of_np
    seed = 81
    b = synth.adversarial_batch(50000, 8, 3, 5000, seed, zipf=0)
    dev = {k: torch.from_numpy(v.view(np.int64) if v.dtype == np.uint64 else
                               (v.view(np.int32) if v.dtype == np.uint32 else v)).cuda() for k, v in b.items()}
    e = engine(synth.adversarial_schema(3), cap=50000, sites=synth.site_ids(8, seed))
    parts, counts = e.partition(dev, nranks)
    dest = rank_of_np(b["table_cid"], b["pk"], nranks)
    order = np.argsort(dest, kind="stable")
    assert counts == np.bincount(dest, minlength=nranks).tolist()
    for k, v in b.items():
        got = parts[k].cpu().numpy().view(v.dtype)
        assert np.array_equal(got, v[order]), k


def test_config1_cpu_reference_workload():
    """BASELINE configs[0]: 100k changes from 4 actors into one 3-column table, pk in [1, 10k]."""
    sites = synth.site_ids(4, synth.config_seed(1))
    b = synth.uniform_batch(100_000, 4, 10_000, 3, synth.config_seed(1), per_version=50)
    e = engine(SCHEMA_T, cap=100_000, sites=sites)
    f = O.Fold(sites)
    assert np.array_equal(e.apply(b, impact=True), f.apply(b))
    compare(e, f)


@pytest.mark.slow
def test_config5_adversarial_scaled():
    """BASELINE configs[4] shape at 1M changes: 8 tables, Zipf(1.1) pks over 2^20, 30 % sentinel
    deletes/resurrects, mixed INTEGER/REAL/TEXT/NULL + 16-byte BLOB values, 1000 actors."""
    seed = synth.config_seed(5)
    sites = synth.site_ids(1000, seed)
    b = synth.adversarial_batch(1_000_000, 1000, 8, 1 << 20, seed)
    e = engine(synth.adversarial_schema(8), cap=1_000_000, sites=sites)
    f = O.Fold(sites)
    e.apply(b)
    f.apply(b)
    compare(e, f, with_ts=True)


@pytest.mark.slow
def test_config2_distribution_4m_vs_oracle():
    """Config 2's distribution (1000 actors, 4 cols, pk space 2^22) at 4M changes, device input."""
    import torch
    seed = synth.config_seed(2)
    sites = synth.site_ids(1000, 1)
    b = synth.uniform_batch(1 << 22, 1000, 1 << 22, 4, seed)
    dev = {k: torch.from_numpy(v.view(np.int64) if v.dtype == np.uint64 else
                               (v.view(np.int32) if v.dtype == np.uint32 else v)).cuda() for k, v in b.items()}
    e = engine({"t": ["a", "b", "c", "d"]}, cap=1 << 22, sites=sites)
    f = O.Fold(sites)
    e.apply(dev)
    f.apply(b)
    compare(e, f)


@pytest.mark.parametrize("n,npk,seed", [(3000, 200, 31), (60000, 9000, 32), (400000, 100000, 33)])
def test_uniform_cl1_impacts_fast_path_vs_oracle(n, npk, seed):
    """cl = 1 batches with impact output take the fast body's member-walk variant (not the
    sequential body): per-change crsql_rows_impacted growth and the merged state must match the
    oracle, across batches (prior state as the first member of a cell)."""
    sites = synth.site_ids(16, seed)
    e = engine({"t": ["a", "b", "c", "d"]}, cap=n, sites=sites)
    f = O.Fold(sites)
    for k in range(3):
        b = synth.uniform_batch(n, 16, npk, 4, seed * 10 + k)
        assert np.array_equal(e.apply(b, impact=True), f.apply(b))
    compare(e, f)


def test_wide_cl1_impacts_fast_path_vs_oracle():
    """Mixed value classes (INTEGER/REAL/TEXT/BLOB/NULL), every cl = 1, no sentinel: the wide fast
    body with impact output, several batches."""
    seed = 34
    sites = synth.site_ids(8, seed)
    e = engine(synth.adversarial_schema(2), cap=40000, sites=sites)
    f = O.Fold(sites)
    for k in range(3):
        b = synth.adversarial_batch(40000, 8, 2, 3000, seed + k, zipf=0, sentinel_frac=0.0, max_cl=1)
        assert np.array_equal(e.apply(b, impact=True), f.apply(b))
    compare(e, f, with_ts=True)


def test_device_batch_device_impacts_vs_oracle():
    """Device-resident batch with impact output: the flags land in a device tensor (no copy)."""
    import torch
    seed = 35
    sites = synth.site_ids(16, seed)
    e = engine({"t": ["a", "b", "c", "d"]}, cap=200000, sites=sites)
    f = O.Fold(sites)
    for k in range(2):
        b = synth.uniform_batch(200000, 16, 30000, 4, seed + k)
        dev = {key: torch.from_numpy(v.view(np.int64) if v.dtype == np.uint64 else
                                     (v.view(np.int32) if v.dtype == np.uint32 else v)).cuda() for key, v in b.items()}
        imp = e.apply(dev, impact=True)
        assert imp.is_cuda and imp.dtype == torch.uint8
        assert np.array_equal(imp.cpu().numpy(), f.apply(b))
    compare(e, f)


@pytest.mark.parametrize("malformed", [False, True])
@pytest.mark.parametrize("impact", [False, True])
def test_parallel_row_fold_overflow_vs_oracle(malformed, impact):
    """Overflow buckets run the parallel row fold (segmented scans over the row's changes, a walk
    over its records only); rows outside App. A.3 (malformed) keep the sequential fold in the same
    bucket. Zipf-hot rows with up to 12 causal-length epochs, several batches (prior state as a
    prefix), impacts on and off."""
    seed = 71 + (2 if malformed else 0) + (1 if impact else 0)
    sites = synth.site_ids(8, seed)
    e = engine(synth.adversarial_schema(3), cap=64, sites=sites)  # one bucket: everything overflows
    f = O.Fold(sites)
    for k in range(3):
        b = synth.adversarial_batch(30000, 8, 3, 300, seed * 10 + k, zipf=1.1, malformed=malformed, max_cl=12)
        got = e.apply(b, impact=impact)
        ref = f.apply(b)
        if impact:
            assert np.array_equal(got, ref), f"impacts differ in batch {k}"
    compare(e, f, with_ts=True)


@pytest.mark.slow
def test_config2_full_size_vs_sharded_oracle():
    """Config 2 at its full size (2^26 changes, pk space 2^22, 1000 actors) generated in HBM, with
    impact flags: all 2^26 impacts equal, rows equal through the order-independent digest of every
    output field, db_versions equal (checker: the oracle's pk-sharded fold on the host cores).
    tools/parity_scale.py runs the same check at 2^29 changes (profiles/history/r01_parity_512m.json)."""
    import torch
    sites = synth.site_ids(1000, 1)
    b = synth.uniform_batch_torch(1 << 26, 1000, 1 << 22, 4, seed=synth.config_seed(2), device="cuda")
    e = engine({"t": ["a", "b", "c", "d"]}, cap=1 << 26, sites=sites)
    imp = e.apply(b, impact=True).cpu().numpy()
    hb = {k: v.cpu().numpy() for k, v in b.items()}
    del b
    torch.cuda.empty_cache()
    for k in ("table_cid", "cl", "seq", "site"):
        hb[k] = hb[k].view(np.uint32)
    for k in ("pk", "val0"):
        hb[k] = hb[k].view(np.uint64)
    f = O.ShardedFold(sites, nshards=64, nthreads=16)
    ref = f.apply(hb)
    assert np.array_equal(imp, ref)
    assert O.rows_digest(e.export()) == f.digest()
    assert np.array_equal(e.db_versions(), f.db_versions())
    e.close()


@pytest.mark.parametrize("cap,chunk", [(64, None), (1 << 12, None), (1 << 12, "65536")])
def test_overflow_fold_mixed_buckets_vs_oracle(monkeypatch, cap, chunk):
    """The device-wide overflow fold against the oracle: every bucket oversized (cap 64), a few
    Zipf-hot buckets among fast ones (cap 4096), chunked applies; malformed rows, mixed value
    classes, impacts, a prior state."""
    if chunk:
        monkeypatch.setenv("CORRO_HIP_CHUNK", chunk)
    seed = 91 + cap % 7 + (3 if chunk else 0)
    sites = synth.site_ids(8, seed)
    e = engine(synth.adversarial_schema(3), cap=cap, sites=sites)
    f = O.Fold(sites)
    for k in range(3):
        b = synth.adversarial_batch(150000, 8, 3, 4000, seed * 10 + k, zipf=1.1, malformed=k == 1, max_cl=12)
        if k == 2:
            e.apply(b)
            f.apply(b)
        else:
            assert np.array_equal(e.apply(b, impact=True), f.apply(b)), f"impacts differ in batch {k}"
        compare(e, f, with_ts=True)


@pytest.mark.parametrize("impact", [False, True])
def test_chunked_apply_equals_one_apply(monkeypatch, impact):
    """A batch larger than the merge's chunk is applied as consecutive chunks in application order:
    the left fold makes that the same result as one apply (forced here with a 4096-change chunk)."""
    monkeypatch.setenv("CORRO_HIP_CHUNK", "4096")
    seed = 61
    sites = synth.site_ids(8, seed)
    b = synth.adversarial_batch(50000, 8, 2, 700, seed)
    e = engine(synth.adversarial_schema(2), cap=50000, sites=sites)
    f = O.Fold(sites)
    got = e.apply(b, impact=impact)
    want = f.apply(b)
    if impact:
        assert np.array_equal(got, want)
    compare(e, f, with_ts=True)


def test_chunked_apply_validates_before_the_first_chunk(monkeypatch):
    """An error in the LAST chunk of a chunked apply leaves the state as it was: the whole batch is
    validated before any chunk commits."""
    import corrosion_amd as ca
    monkeypatch.setenv("CORRO_HIP_CHUNK", "4096")
    seed = 62
    sites = synth.site_ids(8, seed)
    e = engine(synth.adversarial_schema(1), cap=1 << 14, sites=sites)
    e.apply(synth.adversarial_batch(3000, 8, 1, 300, seed))
    before = rows_to_tuples(e.export(), with_ts=True)
    dv = list(e.db_versions())
    b = synth.adversarial_batch(20000, 8, 1, 300, seed + 1)
    b["table_cid"] = b["table_cid"].copy()
    b["table_cid"][-1] = 7  # cid 7 of table 0 does not exist
    with pytest.raises(ca.CorroError) as ex:
        e.apply(b)
    assert ex.value.code == -5
    assert rows_to_tuples(e.export(), with_ts=True) == before
    assert list(e.db_versions()) == dv


@pytest.mark.parametrize("wide", [False, True])
def test_fast_path_folds_into_prior_state(wide):
    """cl=1 batches applied one after another into a growing state (the in-place row store): every
    cell's prior clock is compared with the batch winner, impacts count the prior as the earliest
    member of the cell; alternating impact / no-impact applies, INTEGER and mixed value classes."""
    seed = 81
    sites = synth.site_ids(16, seed)
    e = engine({"t": ["a", "b", "c", "d"]}, cap=40000, sites=sites)
    f = O.Fold(sites)
    for k in range(6):
        b = synth.uniform_batch(40000, 16, 6000, 4, seed + k)
        if wide and k % 3 == 2:  # some TEXT / REAL values (the mixed-class fast bodies)
            rng = np.random.default_rng(seed + k)
            m = rng.random(len(b["pk"])) < 0.3
            b["val_type"] = np.where(m, np.uint8(3), np.uint8(1)).astype(np.uint8)
            b["val_len"] = np.where(m, np.uint8(5), np.uint8(0)).astype(np.uint8)
            b["val1"] = np.zeros(len(b["pk"]), np.uint64)
            # 5-byte TEXT: big-endian bytes in val0, zero padded
            b["val0"] = np.where(m, b["val0"] & np.uint64(0xFFFFFFFFFF000000), b["val0"]).astype(np.uint64)
        if k % 2:
            assert np.array_equal(e.apply(b, impact=True), f.apply(b))
        else:
            e.apply(b)
            f.apply(b)
        compare(e, f)


def test_store_growth_defers_and_regrows():
    """A state far larger than the capacity hint: buckets whose region or the heap cannot take their
    new rows defer before writing, the row store grows, the deferred buckets merge again --
    bit-exact rows and impacts (fast bodies, chunked applies)."""
    seed = 83
    sites = synth.site_ids(16, seed)
    e = engine({"t": ["a", "b", "c", "d"]}, cap=1 << 16, sites=sites)
    f = O.Fold(sites)
    b = synth.uniform_batch(150000, 16, 30000, 4, seed)
    assert np.array_equal(e.apply(b, impact=True), f.apply(b))
    compare(e, f)
    b = synth.uniform_batch(150000, 16, 90000, 4, seed + 1)
    e.apply(b)
    f.apply(b)
    compare(e, f)


def test_general_path_grows_regions():
    """The same growth through the general and overflow bodies (sentinels, Zipf-hot rows)."""
    seed = 84
    sites = synth.site_ids(8, seed)
    e = engine(synth.adversarial_schema(2), cap=1 << 12, sites=sites)
    f = O.Fold(sites)
    for k in range(3):
        b = synth.adversarial_batch(60000, 8, 2, 20000, seed + k, zipf=0.6)
        assert np.array_equal(e.apply(b, impact=True), f.apply(b))
        compare(e, f, with_ts=True)


@pytest.mark.parametrize("cv_max,tie_frac", [(8, 0.5), ((1 << 15) - 1, 0.125), (1 << 15, 0.125), (1 << 40, 0.125)])
def test_fast_body_argmax_forms_vs_oracle(cv_max, tie_frac):
    """The INTEGER fast body without impacts takes the two-stage packed argmax while every
    col_version of the batch is below 2^15 and the three-stage one otherwise (k_scatter's MISC_CVBIG
    flag); both forms, value ties and col_version ties included, against the oracle over a fold."""
    sites = synth.site_ids(40, 5)
    e = engine({"t": ["a", "b", "c", "d"]}, cap=200000, sites=sites)
    f = O.Fold(sites)
    for k in range(3):
        b = synth.uniform_batch(200000, 40, 20000, 4, 900 + k, cv_max=cv_max, tie_frac=tie_frac)
        if cv_max > 8:  # col_version ties as well
            b["col_version"][::3] = cv_max
        e.apply(b)
        f.apply(b)
    compare(e, f)
