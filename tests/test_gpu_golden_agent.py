"""The reference's own end-to-end agent tests, replayed from tests/golden/agent_kats.json (written by
tests/golden/make_golden.py) through the GPU agent:

  * process_failed_changes (/root/reference/crates/corro-agent/src/agent/tests.rs:877-999): the
    version holding an unknown column is rolled back alone, ta2's five versions land with
    crsql_changes db_version = i and site_id = ta2 for pk i (:970-992), no row 6 (:994-998);
  * test_handle_need (/root/reference/crates/corro-agent/src/api/peer/mod.rs:1729-2321): the same
    process_multiple_changes calls, then every handle_need with the messages the reference test
    receives, in order (full needs over overwritten versions, partial needs, the 30-change `wide`
    version that arrives as ten partial changesets and is served from the buffered changes, since
    nothing applies it, empties)."""
import pytest

from tests._util import load_golden

pytestmark = pytest.mark.gpu

SCHEMA = {"tests": ["text"], "tests2": ["text"], "tests3": ["text", "text2", "num", "num2"],
          "testsblob": ["text"], "testsbool": ["b"], "wide": ["int", "float", "blob"]}
INTERNED = ("testsblob", "wide")
K = load_golden("agent_kats.json")


def _val(v):
    t = v["t"]
    if t == "int":
        return int(v["v"])
    if t == "real":
        return float(v["v"])
    if t == "text":
        return v["v"]
    if t == "blob":
        return bytes.fromhex(v["v"])
    return None


def _pk(p):
    if isinstance(p, int):
        return p
    from tests.test_gpu_pk import _pack
    return _pack([bytes.fromhex(c) if isinstance(c, str) else (c["text"] if isinstance(c, dict) else c)
                  for c in p["pack"]])


def _change(c, actor):
    from corrosion_amd.agent import Change
    table, pk, cid, val, cv, dbv, seq, cl = c
    return Change(table, _pk(pk), cid, _val(val), cv, dbv, seq, actor, cl)


def _msg(m, actor, ts):
    from corrosion_amd.agent import ChangeV1, Empty, Full
    if m["kind"] == "empty":
        return ChangeV1(actor, Empty(versions=tuple(m["versions"]), ts=None))
    return ChangeV1(actor, Full(m["version"], [_change(c, actor) for c in m["changes"]], tuple(m["seqs"]),
                                m["last_seq"], ts=ts))


def test_process_failed_changes_fixture():
    from corrosion_amd.agent import Agent, ChangeV1, Full
    f = K["process_failed_changes"]
    ta2, bad = bytes.fromhex(f["ta2"]), bytes.fromhex(f["bad_actor"])
    a = Agent(SCHEMA, capacity_hint=1 << 12, interned=INTERNED)
    msgs = [ChangeV1(bad, Full(f["bad"]["version"], [_change(c, bad) for c in f["bad"]["changes"]],
                               tuple(f["bad"]["seqs"]), f["bad"]["last_seq"]))]
    msgs += [ChangeV1(ta2, Full(g["version"], [_change(c, ta2) for c in g["changes"]], tuple(g["seqs"]),
                                g["last_seq"])) for g in f["good"]]
    r = a.process_multiple_changes(msgs)
    assert r.known[1:] == ["current"] * 5 and r.known[0] not in ("current", "partial")
    rows = a.engine.export()
    site = a.site(ta2)
    got = {int(rows["pk"][i]): (int(rows["db_version"][i]), int(rows["site"][i]))
           for i in range(len(rows["pk"])) if rows["table_cid"][i] >> 16 == 0}
    for pk, dbv in f["expect_dbv"].items():
        assert got[int(pk)] == (dbv, site)
    for pk in f["expect_absent"]:
        assert pk not in got


def test_handle_need_fixture():
    from corrosion_amd.agent import Agent
    from corrosion_amd.sync import Full as NFull, Partial as NPartial
    h = K["handle_need"]
    actor, ts = bytes.fromhex(h["actor"]), h["ts"]
    a = Agent(SCHEMA, capacity_hint=1 << 12, interned=INTERNED)
    for st in h["steps"]:
        if "process" in st:
            r = a.process_multiple_changes([_msg(m, actor, ts) for m in st["process"]])
            assert all(k in ("current", "partial") for k in r.known), r.known
            # (a version completed by partial changesets stays buffered: the reference test never
            # runs process_fully_buffered_changes, so handle_need serves it from the buffer)
            continue
        n = st["need"]
        need = NFull(*n["full"]) if "full" in n else NPartial(n["partial"], tuple(tuple(s) for s in n["seqs"]))
        got = a.handle_needs([(actor, need)])[0]
        if "expect" in st:
            assert got == [_msg(m, actor, ts) for m in st["expect"]], n
        else:
            exp = [_msg(m, actor, ts) for m in st["expect_prefix"]]
            assert got[:len(exp)] == exp, n


def test_clear_empty_versions_fixture():
    """test_clear_empty_versions (agent/tests.rs:777-875) in-process: ta1's 61 versions land in its own
    agent (its bookie books them, as local writes do); ta2 processes 1..=50, then 51..=60; the first
    check_bookie_versions (1..=50 complete: not needed, no gap; no partial); then the sync: ta2's
    generate_sync against ta1's, compute_available_needs on the GPU, ta1's handle_need serving those
    needs from its state, and ta2's process_multiple_changes of what it sent; the second check: no row
    of site ta1 in ta2's crsql_changes at the cleared versions."""
    from corrosion_amd.agent import Agent, ChangeV1, Full
    f = K["clear_empty_versions"]
    ta1, ta2 = bytes.fromhex(f["ta1"]), bytes.fromhex(f["ta2"])
    vers = {v["version"]: v for v in f["ta1_versions"]}

    def msg(v):
        x = vers[v]
        return ChangeV1(ta1, Full(v, [_change(c, ta1) for c in x["changes"]], tuple(x["seqs"]), x["last_seq"],
                                  ts=f["ts"]))
    a1 = Agent(SCHEMA, capacity_hint=1 << 12, actor_id=ta1, interned=INTERNED)
    a2 = Agent(SCHEMA, capacity_hint=1 << 12, actor_id=ta2, interned=INTERNED)
    r = a1.process_multiple_changes([msg(v) for v in sorted(vers)])
    assert r.known == ["current"] * len(vers)
    for s, e in f["calls"]:
        r = a2.process_multiple_changes([msg(v) for v in range(s, e + 1)])
        assert r.known == ["current"] * (e - s + 1)
    ac = f["after_calls"]
    assert a2.bookie.last(ta1) == ac["last"] and a2.bookie.needed(ta1) == [tuple(g) for g in ac["gaps"]]
    for s, e in ac["complete"]:
        assert a2.bookie.contains_all(ta1, (s, e), (0, 3))
        assert all(a2.bookie.partial(ta1, v) is None for v in range(s, e + 1))
    ours, theirs = a2.generate_sync(), a1.generate_sync()
    needs = ours.compute_available_needs(theirs, a2.engine)
    from corrosion_amd.sync import Full as NFull
    assert needs == {ta1: [NFull(s, e) for _k, s, e in f["sync_needs"]]}
    served = a1.handle_needs([(ta1, n) for n in needs[ta1]])
    r = a2.process_multiple_changes([m for msgs in served for m in msgs])
    assert r.known and all(k == "current" for k in r.known)
    rows = a2.engine.export()
    site = a2.site(ta1)
    dbv = {int(rows["db_version"][i]) for i in range(len(rows["pk"])) if int(rows["site"][i]) == site}
    for s, e in f["cleared"]:
        assert not dbv & set(range(s, e + 1)), (s, e, sorted(dbv & set(range(s, e + 1))))
    assert max(dbv) == 61 and a2.bookie.last(ta1) == 61 and a2.bookie.needed(ta1) == []
