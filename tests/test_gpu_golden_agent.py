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
