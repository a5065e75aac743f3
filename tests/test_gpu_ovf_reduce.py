"""GPU parity of the overflow fold's row reduction (ovf_kernels.h, k_ovf_lookup's comment) at its edges,
against the sequential oracle (oracle/crsql_fold.c): the cid mask's last bit (cid 31, tables of 32
columns: reduction on), tables of more columns (reduction off for the batch), and a hot-row batch folded
into a prior state whose rows hold cids the new batch does not touch (rows that must keep every change)."""
import numpy as np
import pytest

import synth
from oracle import oracle as O
from tests._util import rows_to_tuples

pytestmark = pytest.mark.gpu


def _engine(schema, sites, cap=64):
    import corrosion_amd as ca
    e = ca.MergeEngine(schema, capacity_hint=cap)  # a small capacity: every bucket overflows
    e.register_sites(sites)
    return e


def _recid(b, ncols, seed, lo=1):
    """b with its column changes spread over cids lo..ncols (sentinels keep cid 0)"""
    rng = np.random.default_rng(seed)
    tc = np.asarray(b["table_cid"], np.uint32)
    cid = tc & 0xFFFF
    new = rng.integers(lo, ncols + 1, size=len(tc)).astype(np.uint32)
    out = dict(b)
    out["table_cid"] = np.where(cid != 0, (tc & 0xFFFF0000) | new, tc).astype(np.uint32)
    return out


def _compare(e, f):
    assert rows_to_tuples(e.export(), with_ts=True) == rows_to_tuples(f.export(), with_ts=True)
    assert list(e.db_versions()[:f.nsites]) == list(f.db_versions())


def _apply(e, f, b, impact):
    if impact:
        got = e.apply(b, impact=True)
        want = f.apply(b)
        assert np.array_equal(got, want), np.flatnonzero(got != want)[:10]
    else:
        e.apply(b)
        f.apply(b)


@pytest.mark.parametrize("impact", [False, True])
@pytest.mark.parametrize("ncols,lo", [(31, 25), (40, 28)], ids=["cid31_reduced", "wide_not_reduced"])
def test_reduction_cid_mask_edges(ncols, lo, impact):
    seed = 901 + ncols
    sites = synth.site_ids(8, seed)
    e, f = _engine({"t0": [f"c{i}" for i in range(ncols)]}, sites), O.Fold(sites)
    for k in range(3):
        b = _recid(synth.adversarial_batch(40000, 8, 1, 80, seed * 10 + k, zipf=1.1), ncols, seed + k, lo=lo)
        _apply(e, f, b, impact)
    _compare(e, f)


@pytest.mark.parametrize("impact", [False, True])
def test_reduction_keeps_rows_with_untouched_prior_cids(impact):
    """Prior rows hold cids 1..4; the hot batch then only writes cids 1..2 at its largest cl, so rows
    whose prior cells of cids 3..4 are not covered keep every change (and carry those cells)."""
    seed = 933
    sites = synth.site_ids(8, seed)
    e, f = _engine(synth.adversarial_schema(2), sites), O.Fold(sites)
    b1 = synth.adversarial_batch(30000, 8, 2, 200, seed, zipf=1.1)
    b2 = _recid(synth.adversarial_batch(50000, 8, 2, 200, seed + 1, zipf=1.1), 2, seed + 2)
    for b in (b1, b2, b1):
        _apply(e, f, b, impact)
        _compare(e, f)


@pytest.mark.parametrize("max_cl,sent,wide", [(6, 0.3, True), (7, 0.3, False), (3, 0.6, True), (12, 0.3, False),
                                              (5, 0.1, True)])
def test_reduction_impact_form_vs_oracle(max_cl, sent, wide):
    """The impact form of the reduction (k_ovf_keep's comment): a dropped change's flag from its row's
    causal-length slots -- records, no-ops, and candidates by a running argmax over their (row, cl,
    cid) group seeded by a same-cid epoch record -- against the sequential oracle's
    crsql_rows_impacted() growth, three batches folded (prior records in the slots too); with max_cl 12
    many rows hold causal lengths that share a slot (cl mod 8: 1 and 9, ...; those rows keep every
    change)."""
    seed = 950 + max_cl
    sites = synth.site_ids(12, seed)
    e, f = _engine(synth.adversarial_schema(3), sites), O.Fold(sites)
    for k in range(3):
        b = synth.adversarial_batch(60000, 12, 3, 96, seed * 10 + k, zipf=1.1, max_cl=max_cl, sentinel_frac=sent,
                                    wide=wide)
        _apply(e, f, b, True)
        _compare(e, f)


def _tie_batch(n, npk, sites_n, seed, dbv0=1, cl_max=3):
    """Hot rows whose changes at the largest causal length tie on (col_version, value, site) in every
    cell: only db_version / seq / ts tell them apart, so the winner must be the earliest change."""
    rng = np.random.default_rng(seed)
    i = np.arange(n, dtype=np.int64)
    pk = rng.integers(1, npk + 1, size=n).astype(np.uint64)
    site = rng.integers(0, sites_n, size=n).astype(np.uint32)
    cid = rng.integers(1, 5, size=n).astype(np.uint32)
    cl = (2 * rng.integers(0, (cl_max + 1) // 2, size=n) + 1).astype(np.uint32)  # odd: column changes
    cv = np.full(n, 3, np.int64)
    v0 = np.full(n, 7, np.uint64)
    dbv = (dbv0 + i // 16).astype(np.int64)
    seq = (i % 16).astype(np.uint32)
    vt = np.full(n, 1, np.uint8)
    return {"pk": pk, "table_cid": cid, "col_version": cv, "db_version": dbv, "cl": cl, "seq": seq, "site": site,
            "val0": v0, "val1": np.zeros(n, np.uint64), "val_type": vt, "val_len": np.zeros(n, np.uint8),
            "ts": (dbv.astype(np.uint64) << np.uint64(20)) + site.astype(np.uint64)}


def test_reduced_cells_settle_exact_ties_by_position():
    """Round 6's fused plain fold: a reduced row's cells are sorted by (owner record, cid) only, so the
    sort's order inside a cell is not the application order and exact ties -- equal col_version, value
    and site -- are settled by the position tie-break of the argmax (the earliest change wins, its
    db_version / seq / ts kept). Two batches: the second ties against the prior clocks too (a prior
    record comes first in application order)."""
    seed = 977
    sites = synth.site_ids(2, seed)
    e, f = _engine({"t0": list(synth.ADV_COLS)}, sites), O.Fold(sites)
    for k, dbv0 in enumerate((1, 100000)):
        b = _tie_batch(30000, 40, 1 if k else 2, seed + k, dbv0=dbv0)
        _apply(e, f, b, False)
        _compare(e, f)
