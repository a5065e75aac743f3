"""Pin the CPU oracle against the reference's own known-answer vectors (no GPU)."""
import numpy as np
import pytest

from oracle import oracle as O
from tests._util import batch_from_changes, expected_rows, load_golden, rows_to_tuples, site_table
from tests.sync_util import decode_needs, entries_from_pairs, kat_expect

MERGE = load_golden("merge_kats.json")


@pytest.mark.parametrize("case", MERGE["cases"], ids=[c["name"][:3] for c in MERGE["cases"]])
def test_oracle_merge_kats(case):
    f = O.Fold(site_table())
    imp = f.apply(batch_from_changes(case["changes"]))
    got = [t[:11] for t in rows_to_tuples(f.export())]
    assert got == expected_rows(case["rows"])
    assert list(np.cumsum(imp)) == case["impacted"]


def test_oracle_db_versions():
    c = MERGE["db_versions_case"]
    f = O.Fold(site_table())
    f.apply(batch_from_changes(c["changes"]))
    dv = f.db_versions()
    for site, v in c["db_versions"].items():
        assert dv[int(site)] == v
    assert dv[0] == -1


def test_oracle_merge_kats_as_one_batch_over_many_pks():
    """All KATs at once, each on its own pk, interleaved: per-pk results must not change."""
    f = O.Fold(site_table())
    parts, exp = [], []
    for i, case in enumerate(MERGE["cases"]):
        parts.append(batch_from_changes(case["changes"], pk=100 + i))
        exp += expected_rows(case["rows"], pk=100 + i)
    # interleave round-robin, keeping per-pk order
    order = []
    idx = [0] * len(parts)
    while any(idx[j] < len(parts[j]["pk"]) for j in range(len(parts))):
        for j in range(len(parts)):
            if idx[j] < len(parts[j]["pk"]):
                order.append((j, idx[j]))
                idx[j] += 1
    batch = {k: np.array([parts[j][k][i] for j, i in order], dtype=parts[0][k].dtype) for k in parts[0]}
    f.apply(batch)
    assert [t[:11] for t in rows_to_tuples(f.export())] == sorted(exp)


SYNC = load_golden("sync_kats.json")


@pytest.mark.parametrize("case", SYNC["cases"], ids=[c["name"] for c in SYNC["cases"]])
def test_oracle_sync_kats(case):
    ent = entries_from_pairs([(case["our"], case["their"])])
    res = O.needs(ent)
    assert decode_needs(res, 1)[0] == kat_expect(case["expect"])


def test_oracle_gaps_kats():
    steps = load_golden("gaps_kats.json")["steps"]
    b, allv = O.Booked(), []
    for st in steps:
        if st.get("reset"):
            b, allv = O.Booked(), []
            continue
        assert b.insert_db(st["insert"]) == 0
        allv += st["insert"]
        if st["gaps"] is not None:
            assert b.needed() == [tuple(g) for g in st["gaps"]]
            for s, e in st["gaps"]:
                for v in range(s, e + 1):
                    assert not b.contains(v)
        for s, e in allv:
            for v in range(s, e + 1):
                if st["gaps"] is not None and any(gs <= v <= ge for gs, ge in st["gaps"]):
                    continue
                assert b.contains(v)
        assert b.max() == max(e for _, e in allv)


@pytest.mark.parametrize("nshards,nthreads", [(1, 1), (7, 3), (16, 8)])
def test_sharded_fold_equals_sequential_fold(nshards, nthreads):
    """The pk-sharded parallel fold (CPU baseline / 512M checker) reproduces the sequential fold:
    same impacts, same rows (digest and exported rows), same crsql_db_versions."""
    import synth
    sites = synth.site_ids(8, 3)
    batches = [synth.adversarial_batch(30000, 8, 2, 400, 11), synth.uniform_batch(30000, 8, 500, 4, 12),
               synth.adversarial_batch(20000, 8, 2, 400, 13, malformed=True)]
    f = O.Fold(sites)
    g = O.ShardedFold(sites, nshards=nshards, nthreads=nthreads)
    for b in batches:
        assert np.array_equal(f.apply(b), g.apply(b))
    assert g.digest() == O.rows_digest(f.export())
    assert np.array_equal(g.db_versions(), f.db_versions())


def test_rows_digest_detects_a_single_field_change():
    import synth
    f = O.Fold(synth.site_ids(4, 1))
    f.apply(synth.uniform_batch(5000, 4, 300, 4, 3))
    rows = f.export()
    d0 = O.rows_digest(rows)
    perm = np.random.default_rng(0).permutation(len(rows["pk"]))
    rows.pop("long_values")
    assert O.rows_digest({k: v[perm] for k, v in rows.items()}) == d0  # order-independent
    for k in rows:
        r2 = {kk: vv.copy() for kk, vv in rows.items()}
        r2[k][17] ^= 1
        assert O.rows_digest(r2) != d0, k


def test_needs_parallel_equals_needs():
    """The threaded chunked need diff (the full-size config-4 checker) equals the single pass."""
    from tests.sync_util import entries_from_pairs
    from tests.test_gpu_sync import random_side
    rng = np.random.default_rng(17)
    pairs = [(random_side(rng, with_head=rng.random() < 0.9), random_side(rng)) for _ in range(3000)]
    ent = entries_from_pairs(pairs)
    a = O.needs(ent)
    b = O.needs_parallel(ent, nthreads=4, chunk=257)
    for k in a:
        assert np.array_equal(a[k], b[k]), k


def test_inverted_our_need_ranges_fixture():
    """Entries whose our-need list holds an inverted (empty) range, as a peer's message could:
    the oracle keeps rangemap's overlapping() semantics (a have range spanning [t, s] yields
    Full(s..=t)); the fixture pins that output for the GPU test."""
    from tests.sync_util import decode_needs, entries_from_pairs, expected_from_cases, pairs_from_cases
    cases = load_golden("sync_inverted_cases.json")["cases"]
    ent = entries_from_pairs(pairs_from_cases(cases))
    assert decode_needs(O.needs(ent), len(cases)) == expected_from_cases(cases)


LONG_POOL = ["v0", "same-prefix", "same-pre", "same-prefix-and-then-some", "same-prefix-and-then-somf",
             "same-prefix-and-then-some-more", "0123456789abcdef", "0123456789abcdef0", "x" * 300,
             b"\0" * 16, b"\0" * 17, b"\0" * 40, b"\0" * 16 + b"\1", bytes(range(64))]


def _value_key(v):
    """SQLite value order for TEXT/BLOB (memcmp, then length): Python's bytes order; TEXT > BLOB."""
    return (1 if isinstance(v, str) else 0, v.encode() if isinstance(v, str) else bytes(v))


def test_oracle_long_values_lww_order():
    """Values of any length (SqliteValue::Text / Blob, corro-api-types/src/lib.rs:419-429): at equal
    col_version the greater value wins by memcmp-then-length over the WHOLE value (not a 16-byte
    prefix), and the state keeps every byte."""
    from tests._util import encode_values
    rng = np.random.default_rng(11)
    n = 4000
    vals = [LONG_POOL[int(rng.integers(0, len(LONG_POOL)))] for _ in range(n)]
    pks = rng.integers(0, 40, n).astype(np.uint64)
    b = encode_values(vals)
    b.update({"pk": pks, "table_cid": np.ones(n, np.uint32), "col_version": np.ones(n, np.int64),
              "db_version": np.arange(1, n + 1, dtype=np.int64), "cl": np.ones(n, np.uint32),
              "seq": np.zeros(n, np.uint32), "site": (np.arange(n) % 3).astype(np.uint32)})
    f = O.Fold(site_table(4))
    imp = f.apply(b)
    rows = f.export()
    got = {int(rows["pk"][i]): i for i in range(len(rows["pk"]))}
    for pk in range(40):
        mine = [(v, j) for j, v in enumerate(vals) if pks[j] == pk]
        if not mine:
            continue
        # winner: max value; among equal values the larger site id, then the earliest change
        best = max(mine, key=lambda t: (_value_key(t[0]), t[1] % 3, -t[1]))
        i = got[pk]
        v = best[0]
        raw = v.encode() if isinstance(v, str) else bytes(v)
        if len(raw) > 16:
            assert rows["val_len"][i] == O.OF_LONG and rows["long_values"][i] == raw
        else:
            assert rows["val_len"][i] == len(raw)
        assert rows["db_version"][i] == best[1] + 1
    # impacts: strict prefix maxima of (value, site) per pk
    cur = {}
    for j, v in enumerate(vals):
        k = (_value_key(v), j % 3)
        exp = 1 if (int(pks[j]) not in cur or k > cur[int(pks[j])]) else 0
        if exp:
            cur[int(pks[j])] = k
        assert imp[j] == exp, j
    # the digest sees the bytes: a copy of the rows with the same long values digests equal
    assert O.rows_digest(rows)[0] == len(rows["pk"])
    s = O.ShardedFold(site_table(4), nshards=4, nthreads=2)
    s.apply(b)
    assert s.digest() == O.rows_digest(rows)


def test_agent_oracle_empty_set_is_skipped():
    """Changeset::EmptySet through the process_multiple_changes restatement: versions() = 0..=0
    (broadcast.rs:176), contains_version(0) holds with or without a max (agent.rs:1353-1361), so pass
    1 skips it (util.rs:724-733) -- for a fresh actor and for one with bookkeeping alike."""
    import synth
    from oracle.agent import AgentOracle, Changeset
    ids = synth.site_ids(2, 9)
    ref = AgentOracle(ids)
    es = Changeset(ids[0], "empty_set", versions=[(3, 5)], ts=7)
    assert ref.process([es]) == (["skipped"], [[]])
    assert ref.last(bytes(ids[0])) is None and not ref.set_dbv
    full = Changeset(ids[1], "full", version=2, seqs=(0, 0), last_seq=0, ts=1,
                     rows=[dict(pk=1, table_cid=1, col_version=1, db_version=2, cl=1, seq=0, site=1, val0=5)])
    known, _ = ref.process([full, Changeset(ids[1], "empty_set", versions=[(1, 1)])])
    assert known == ["current", "skipped"]
    assert ref.last(bytes(ids[1])) == 2 and ref.needed(bytes(ids[1])) == [(1, 1)]


def _clear_empty_versions_oracle_rows(v, site):
    """a fixture version's changes as oracle rows (tests3 = table 0, columns text/text2/num/num2 =
    cids 1..4; TEXT values as small INTEGER stand-ins: the test asserts bookkeeping and db_versions)"""
    cols = {"text": 1, "text2": 2, "num": 3, "num2": 4}
    out = []
    for _t, pk, col, val, cv, dbv, seq, cl in v["changes"]:
        x = int(val["v"]) if val["t"] == "int" else len(val["v"])
        out.append(dict(pk=pk, table_cid=cols[col], col_version=cv, db_version=dbv, cl=cl, seq=seq, site=site,
                        val0=x & ((1 << 64) - 1), val_type=1))
    return out


def test_clear_empty_versions_fixture_on_the_restatement():
    """test_clear_empty_versions (agent/tests.rs:777-875) through oracle/agent.py: the two calls leave
    1..=50 complete, no gaps, last 60; ta2's sync state against ta1's needs exactly 61..=61 (the
    restated compute_available_needs); after it lands no row of ta1's is left at the cleared versions."""
    from oracle.agent import AgentOracle, Changeset
    f = load_golden("agent_kats.json")["clear_empty_versions"]
    ta1, ta2 = bytes.fromhex(f["ta1"]), bytes.fromhex(f["ta2"])
    ids = np.frombuffer(ta1 + ta2, np.uint8).reshape(2, 16)
    vers = {v["version"]: v for v in f["ta1_versions"]}

    def cs(v):
        x = vers[v]
        return Changeset(ta1, "full", version=v, seqs=tuple(x["seqs"]), last_seq=x["last_seq"], ts=f["ts"],
                         rows=_clear_empty_versions_oracle_rows(x, 0))
    src, dst = AgentOracle(ids), AgentOracle(ids)
    known, _ = src.process([cs(v) for v in sorted(vers)])
    assert known == ["current"] * len(vers)
    for a, b in f["calls"]:
        known, _ = dst.process([cs(v) for v in range(a, b + 1)])
        assert known == ["current"] * (b - a + 1)
    assert dst.last(ta1) == f["after_calls"]["last"] and dst.needed(ta1) == []
    ent = entries_from_pairs([({"head": dst.last(ta1), "need": dst.needed(ta1)},
                               {"head": src.last(ta1), "need": src.needed(ta1)})])
    got = decode_needs(O.needs(ent), 1)[0]
    assert got == [tuple(n) for n in f["sync_needs"]]
    for kind, s, e in got:
        dst.process([cs(v) for v in range(s, e + 1)])
    rows = dst.export()
    dbv = {int(rows["db_version"][i]) for i in range(len(rows["pk"])) if int(rows["site"][i]) == 0}
    for s, e in f["cleared"]:
        assert not dbv & set(range(s, e + 1)), (s, e)
    assert dbv == set(range(1, 62)) - {v for s, e in f["cleared"] for v in range(s, e + 1)} - {31}
