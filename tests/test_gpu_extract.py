"""GPU parity of the sync server's changeset extraction (corro_extract_changes, csrc/extract.hip)
against the oracle restatement of handle_need's two queries (oracle.extract_changes over the
exported crsql_changes rows), and handle_need end to end (corrosion_amd/serve.py) on an agent
state built through process_multiple_changes. Bar: identical versions (DESC), MAX(seq), MAX(ts)
and rows (seq ASC; ties on seq compared as a set, the SQL leaves their order open)."""
import numpy as np
import pytest

import synth
from oracle import oracle as O

pytestmark = pytest.mark.gpu

ROWF = ("pk", "table_cid", "col_version", "db_version", "cl", "seq", "site", "ts", "val0", "val1", "val_type",
        "val_len")


def _rows_tuple(rows, idx):
    t = [tuple(int(rows[k][i]) for k in ROWF) for i in idx]
    return sorted(t, key=lambda r: (r[5], r[1], r[0]))


def got_groups(res, e):
    from corrosion_amd.engine import ROW_FIELDS
    # device results come back as signed torch dtypes: view them in the row field types
    rows = {k: (v.cpu().numpy().view(ROW_FIELDS[k]) if hasattr(v, "cpu") else v) for k, v in res["rows"].items()}
    R = {k: (v.cpu().numpy() if hasattr(v, "cpu") else v) for k, v in res.items() if k != "rows"}
    out = []
    for g in range(int(R["grp_off"][e]), int(R["grp_off"][e + 1])):
        ro, rn = int(R["grp_row_off"][g]), int(R["grp_rows"][g])
        out.append((int(R["version"][g]), int(R["last_seq"][g]), int(R["ts"][g]), _rows_tuple(rows, range(ro, ro + rn))))
    return out


def exp_groups(rows, groups):
    return [(v, last, ts, _rows_tuple(rows, g)) for v, last, ts, g in groups]


def random_needs(rng, n, nsites, max_dbv, seq_filter):
    site = rng.integers(0, nsites + 2, n).astype(np.uint32)       # a few unknown sites
    start = rng.integers(0, max_dbv + 3, n).astype(np.uint64)
    span = rng.integers(0, 6, n)
    end = (start + span.astype(np.uint64)).astype(np.uint64)
    end[::17] = start[::17] - np.uint64(1)                        # some start > end (empty)
    end[::23] = np.uint64(1 << 62)                                 # open-ended
    nd = {"site": site, "start": start, "end": end}
    if seq_filter:
        a = rng.integers(0, 70, n).astype(np.uint32)
        b = (a + rng.integers(0, 20, n)).astype(np.uint32)
        b[::13] = a[::13] - 1                                      # empty seq range
        nd["seq_start"], nd["seq_end"] = a, b
    return nd


def _engine(schema, sites, cap=1 << 16):
    import corrosion_amd as ca
    e = ca.MergeEngine(schema, capacity_hint=cap)
    e.register_sites(sites)
    return e


@pytest.mark.parametrize("kind,seq_filter", [("uniform", False), ("uniform", True), ("adversarial", False),
                                             ("adversarial", True)])
def test_extract_vs_oracle(kind, seq_filter):
    sites = synth.site_ids(8, 3)
    if kind == "uniform":
        schema = {"t": ["a", "b", "c", "d"]}
        b = synth.uniform_batch(60000, 8, 4000, 4, 41)
        b["ts"] = (b["db_version"].astype(np.uint64) << np.uint64(8)) + b["seq"].astype(np.uint64)
    else:
        schema = synth.adversarial_schema(3)
        b = synth.adversarial_batch(60000, 8, 3, 3000, 42)
    e = _engine(schema, sites)
    e.apply(b)
    rows = e.export()
    f = O.Fold(sites)
    f.apply(b)
    assert O.rows_digest(rows) == O.rows_digest(f.export())
    rng = np.random.default_rng(7)
    nd = random_needs(rng, 3000, 8, int(b["db_version"].max()), seq_filter)
    res = e.extract_changes(nd)
    exp = O.extract_changes(rows, nd)
    for i in range(len(nd["site"])):
        assert got_groups(res, i) == exp_groups(rows, exp[i]), i


def test_extract_device_needs_equal_host_needs():
    import torch
    sites = synth.site_ids(8, 3)
    b = synth.uniform_batch(40000, 8, 3000, 4, 43)
    e = _engine({"t": ["a", "b", "c", "d"]}, sites)
    e.apply(b)
    nd = random_needs(np.random.default_rng(8), 2000, 8, int(b["db_version"].max()), True)
    host = e.extract_changes(nd)
    dev = e.extract_changes({k: torch.from_numpy(v.view(np.int64) if v.dtype == np.uint64 else v.view(np.int32)).cuda()
                             for k, v in nd.items()})
    for i in range(0, 2000, 7):
        assert got_groups(dev, i) == got_groups(host, i)


def test_extract_two_sort_path_large_versions():
    """db_version near 2^50 and seq near 2^31: (site, dbv, seq) no longer packs into 64 bits, so the
    index takes two stable radix sorts."""
    sites = synth.site_ids(4, 5)
    b = synth.uniform_batch(20000, 4, 2000, 4, 44)
    b["db_version"] = b["db_version"] + np.int64(1 << 50)
    b["seq"] = (b["seq"].astype(np.uint64) + np.uint64((1 << 31) - 200)).astype(np.uint32)
    e = _engine({"t": ["a", "b", "c", "d"]}, sites)
    e.apply(b)
    rows = e.export()
    lo = int(b["db_version"].min())
    nd = {"site": np.array([0, 1, 2, 3, 1], np.uint32),
          "start": np.array([lo, lo + 3, lo, lo + 40, lo + 1], np.uint64),
          "end": np.array([lo + 5, lo + 3, lo + 100, lo + 41, lo + 1], np.uint64)}
    res = e.extract_changes(nd)
    exp = O.extract_changes(rows, nd)
    for i in range(5):
        assert got_groups(res, i) == exp_groups(rows, exp[i])
    assert sum(len(g) for g in exp) > 0


def test_extract_edge_cases_and_index_refresh():
    sites = synth.site_ids(4, 6)
    e = _engine({"t": ["a", "b", "c", "d"]}, sites)
    nd = {"site": np.array([0, 9], np.uint32), "start": np.array([1, 1], np.uint64),
          "end": np.array([100, 100], np.uint64)}
    res = e.extract_changes(nd)                      # empty state
    assert int(res["grp_off"][-1]) == 0 and int(res["row_off"][-1]) == 0
    b1 = synth.uniform_batch(5000, 4, 500, 4, 45)
    e.apply(b1)
    r1 = e.extract_changes(nd)
    assert got_groups(r1, 1) == []                  # unknown site ordinal
    b2 = synth.uniform_batch(5000, 4, 500, 4, 46)
    b2["db_version"] = b2["db_version"] + 1000
    e.apply(b2)                                      # new state epoch: index rebuilt
    rows = e.export()
    nd2 = {"site": np.array([0, 1, 2, 3], np.uint32), "start": np.array([1, 990, 1000, 0], np.uint64),
           "end": np.array([2000, 1010, 1000, 0], np.uint64)}
    res = e.extract_changes(nd2)
    exp = O.extract_changes(rows, nd2)
    for i in range(4):
        assert got_groups(res, i) == exp_groups(rows, exp[i])
    e.reset()
    assert int(e.extract_changes(nd2)["grp_off"][-1]) == 0


# ---- handle_need end to end --------------------------------------------------------------

def test_handle_need_full_partial_empty_and_buffered():
    from tests.test_gpu_agent import TA1, Node, agent
    from corrosion_amd.agent import ChangeV1, Empty, Full
    from corrosion_amd.sync import Full as NFull, Partial as NPartial
    ta1, b = Node(TA1), agent()
    ta1.insert_rows(1, 12)
    b.process_multiple_changes(ta1.get_rows([((1, 5), None), ((6, 6), (0, 1))]))
    b.process_multiple_changes([ChangeV1(TA1, Empty((7, 7)))])
    exp_full = [ChangeV1(TA1, Full(v, sorted(ta1.rows[v], key=lambda c: c.seq), (0, 3), 3, ts=1000 + v))
                for v in (5, 4, 3, 2, 1)]
    v6 = sorted(ta1.rows[6], key=lambda c: c.seq)[:2]
    got = b.handle_needs([(TA1, NFull(1, 8)), (TA1, NPartial(6, ((0, 1),))), (TA1, NPartial(3, ((1, 2),))),
                          (TA1, NPartial(9, ((0, 3),)))])
    assert got[0] == exp_full + [ChangeV1(TA1, Full(6, v6, (0, 1), 3, ts=1006)), ChangeV1(TA1, Empty((7, 8)))]
    assert got[1] == [ChangeV1(TA1, Full(6, v6, (0, 1), 3, ts=1006))]
    v3 = sorted(ta1.rows[3], key=lambda c: c.seq)[1:3]
    assert got[2] == [ChangeV1(TA1, Full(3, v3, (1, 2), 3, ts=1003))]
    assert got[3] == [ChangeV1(TA1, Empty((9, 9)))]
    # a gap: 11 applied with 8..10 unseen -> 8..10 are needed (skipped), 7 and 12 are empties
    b.process_multiple_changes(ta1.get_rows([((11, 11), None)]))
    got = b.handle_needs([(TA1, NFull(7, 12))])[0]
    assert got == [ChangeV1(TA1, Full(11, sorted(ta1.rows[11], key=lambda c: c.seq), (0, 3), 3, ts=1011)),
                   ChangeV1(TA1, Empty((7, 7))), ChangeV1(TA1, Empty((12, 12)))]


def test_handle_need_chunks_large_versions():
    """A version larger than MAX_CHANGES_BYTES_PER_MESSAGE goes out in seq-contiguous chunks whose
    last one ends at last_seq (ChunkedChanges, change.rs:66-178)."""
    from tests.test_gpu_agent import TA1, agent
    from corrosion_amd import serve
    from corrosion_amd.agent import Change, ChangeV1, Full
    from corrosion_amd.sync import Full as NFull
    b = agent()
    ch = [Change("tests3", 1000 + k, "num", k, 1, 1, k, TA1, 1) for k in range(300)]
    b.process_multiple_changes([ChangeV1(TA1, Full(1, ch, (0, 299), 299, ts=5))])
    got = b.handle_needs([(TA1, NFull(1, 1))])[0]
    exp = [ChangeV1(TA1, Full(1, c, s, 299, ts=5)) for c, s in serve.ChunkedChanges(ch, 0, 299, 8 * 1024)]
    assert len(exp) > 2 and got == exp
    assert sum(len(m.changeset.changes) for m in got) == 300
