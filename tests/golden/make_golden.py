"""Transcribe the reference's known-answer vectors for this path into JSON fixtures.

Run: python tests/golden/make_golden.py   (writes merge_kats.json, sync_kats.json, gaps_kats.json)

Sources (data only, no reference code is copied):
  * merge_kats   — SURVEY.md Appendix A.5 KAT table K1..K18 + its "additional probe facts"
                   (cr-sqlite 0.17.0 results recorded during the survey) and the conflict example in
                   /root/reference/doc/crdts.md:166-245 ('started' beats 'destroyed' at col_version 2).
  * sync_kats    — the four assertions of test_compute_available_needs,
                   /root/reference/crates/corro-types/src/sync.rs:386-500.
  * gaps_kats    — the insert/expect_gaps steps of test_booked_insert_db,
                   /root/reference/crates/corro-types/src/agent.rs:1605-1868.
  * chunker_kats — the cases of test_change_chunker, /root/reference/crates/corro-types/src/change.rs:
                   266-401: Change { seq, ..Default::default() } (empty table/cid/pk, Null value), so
                   every change's estimated_byte_size is the same; max_buf_size is given in changes.
  * agent_kats   — two end-to-end scenarios over corro-tests' TEST_SCHEMA
                   (/root/reference/crates/corro-tests/src/lib.rs:13-53):
                   process_failed_changes, /root/reference/crates/corro-agent/src/agent/tests.rs:
                   877-999 (the bad-cid version rolled back alone; db_version / site of pks 1..5 as
                   asserted at :970-992; pk 6 absent), and test_handle_need,
                   /root/reference/crates/corro-agent/src/api/peer/mod.rs:1729-2321 (every
                   process_multiple_changes call and every handle_need with the messages the test
                   receives, in order). The reference draws the `wide` rows' int / float / blob from
                   rand::thread_rng; fixed stand-ins are recorded here (the assertions compare the
                   served changes with the applied ones, whatever their values). Change notation:
                   [table, pk, cid, value, col_version, db_version, seq, cl], pk = an int (one packed
                   INTEGER) or {"pack": [hex blob | {"text": s} | int, ...]} (pack_columns).

Merge-case notation: table t(id INTEGER PK, a, b, c); cid 0 = sentinel '-1', a=1, b=2, c=3.
Sites sN = sixteen bytes of value N. A change is [cid, value, col_version, db_version, site, cl];
value = {"t": "int"|"real"|"text"|"blob"|"null", "v": ...}. `impacted` is the cumulative
crsql_rows_impacted() after each insert (one transaction).
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))


def I(v):
    return {"t": "int", "v": v}


def R(v):
    return {"t": "real", "v": v}


def T(v):
    return {"t": "text", "v": v}


def B(hexs):
    return {"t": "blob", "v": hexs}


N = {"t": "null", "v": None}
S = 0  # sentinel cid

MERGE = [
    # name, input changes, expected final rows (cid, val, cv, dbv, site, cl), impacted, source
    ("K1 first write cl=1", [[1, I(5), 1, 7, 1, 1]], [[1, I(5), 1, 7, 1, 1]], [1]),
    ("K2 equal colv, bigger value wins", [[1, I(5), 1, 7, 1, 1], [1, I(6), 1, 3, 2, 1]],
     [[1, I(6), 1, 3, 2, 1]], [1, 2]),
    ("K3 equal colv, smaller value loses", [[1, I(6), 1, 3, 2, 1], [1, I(4), 1, 9, 2, 1]],
     [[1, I(6), 1, 3, 2, 1]], [1, 1]),
    ("K4 higher colv beats bigger value", [[1, I(9), 1, 7, 1, 1], [1, I(1), 2, 3, 2, 1]],
     [[1, I(1), 2, 3, 2, 1]], [1, 2]),
    ("K5 equal value+colv: bigger site wins",
     [[1, I(5), 1, 7, 2, 1], [1, I(5), 1, 3, 1, 1], [1, I(5), 1, 4, 3, 1]],
     [[1, I(5), 1, 4, 3, 1]], [1, 1, 2]),
    ("K6 type rank INTEGER > REAL", [[1, R(5.5), 1, 7, 1, 1], [1, I(5), 1, 8, 2, 1]],
     [[1, I(5), 1, 8, 2, 1]], [1, 2]),
    ("K7 REAL loses to INTEGER", [[1, I(5), 1, 7, 1, 1], [1, R(5.5), 1, 8, 2, 1]],
     [[1, I(5), 1, 7, 1, 1]], [1, 1]),
    ("K8 NULL loses", [[1, I(5), 1, 7, 1, 1], [1, N, 1, 8, 2, 1]],
     [[1, I(5), 1, 7, 1, 1]], [1, 1]),
    ("K9 BLOB memcmp", [[3, B("6162"), 1, 7, 1, 1], [3, B("62"), 1, 8, 2, 1]],
     [[3, B("62"), 1, 8, 2, 1]], [1, 2]),
    ("K10 remote delete drops row", [[1, I(5), 1, 1, 1, 1], [S, N, 2, 2, 2, 2]],
     [[S, N, 2, 2, 2, 2]], [1, 2]),
    ("K11 stale col after delete ignored", [[S, N, 2, 2, 2, 2], [1, I(5), 9, 1, 1, 1]],
     [[S, N, 2, 2, 2, 2]], [1, 1]),
    ("K12 resurrect via column after delete",
     [[1, I(5), 4, 1, 1, 1], [S, N, 2, 2, 2, 2], [1, I(7), 1, 3, 3, 3]],
     [[S, N, 3, 3, 3, 3], [1, I(7), 1, 3, 3, 3]], [1, 2, 4]),
    ("K13 missed-delete resurrect zeroes colv", [[1, I(5), 9, 1, 1, 1], [2, I(7), 1, 3, 3, 3]],
     [[S, N, 3, 3, 3, 3], [1, I(5), 0, 1, 1, 3], [2, I(7), 1, 3, 3, 3]], [1, 3]),
    ("K14 same as K13, reversed order", [[2, I(7), 1, 3, 3, 3], [1, I(5), 9, 1, 1, 1]],
     [[S, N, 3, 3, 3, 3], [2, I(7), 1, 3, 3, 3]], [2, 2]),
    ("K15 first write cl=3 creates sentinel", [[1, I(5), 1, 3, 3, 3]],
     [[S, N, 3, 3, 3, 3], [1, I(5), 1, 3, 3, 3]], [2]),
    ("K16 pk-only sentinel cl=1", [[S, N, 1, 2, 2, 1]], [[S, N, 1, 2, 2, 1]], [1]),
    ("K17 sentinel cl=1 after column = no-op", [[1, I(5), 1, 1, 1, 1], [S, N, 1, 2, 2, 1]],
     [[1, I(5), 1, 1, 1, 1]], [1, 1]),
    ("K18 equal delete twice = no-op", [[S, N, 2, 2, 2, 2], [S, N, 2, 5, 3, 2]],
     [[S, N, 2, 2, 2, 2]], [1, 1]),
    ("P1 identical duplicate from the same site: no impact",
     [[1, I(5), 1, 7, 1, 1], [1, I(5), 1, 7, 1, 1]], [[1, I(5), 1, 7, 1, 1]], [1, 1]),
    ("P2 sentinel resurrect cv=7 cl=3 stores sentinel cv 7 (row cl reads 7)",
     [[S, N, 2, 1, 1, 2], [S, N, 7, 2, 2, 3]], [[S, N, 7, 2, 2, 7]], [1, 2]),
    ("D1 doc/crdts.md: 'started' beats 'destroyed' at equal col_version",
     [[1, T("meow"), 1, 1, 5, 1], [2, T("destroyed"), 2, 5, 6, 1], [2, T("started"), 2, 3, 5, 1]],
     [[1, T("meow"), 1, 1, 5, 1], [2, T("started"), 2, 3, 5, 1]], [1, 2, 3]),
    ("D2 doc/crdts.md reverse direction: 'destroyed' loses to 'started'",
     [[1, T("meow"), 1, 1, 5, 1], [2, T("started"), 2, 3, 5, 1], [2, T("destroyed"), 2, 5, 6, 1]],
     [[1, T("meow"), 1, 1, 5, 1], [2, T("started"), 2, 3, 5, 1]], [1, 2, 2]),
]

# crsql_db_versions after {s3 dbv3 applied; s2 dbv17 ignored (cl<L);
# s1 dbv21 lost on value; s4 dbv30 sentinel no-op} = {s1:21, s2:17, s3:3, s4:30}
DBV = {
    "name": "crsql_db_versions records every inserted change, losers included",
    "changes": [[1, I(5), 1, 3, 3, 3], [1, I(9), 5, 17, 2, 1], [1, I(4), 1, 21, 1, 3],
                [S, N, 3, 30, 4, 3]],
    "db_versions": {"1": 21, "2": 17, "3": 3, "4": 30},
}

# sync.rs:386-500 (actor1 heads/needs; one actor)
SYNC = [
    {"name": "heads only", "our": {"head": 10, "need": [], "partials": {}},
     "their": {"head": 13, "need": [], "partials": {}},
     "expect": [["full", 11, 13]]},
    {"name": "our needs inside their haves", "our": {"head": 10, "need": [[2, 5], [7, 7]], "partials": {}},
     "their": {"head": 13, "need": [], "partials": {}},
     "expect": [["full", 2, 5], ["full", 7, 7], ["full", 11, 13]]},
    {"name": "our partial, they have the version",
     "our": {"head": 10, "need": [[2, 5], [7, 7]], "partials": {"9": [[100, 120], [130, 132]]}},
     "their": {"head": 13, "need": [], "partials": {}},
     "expect": [["full", 2, 5], ["full", 7, 7], ["partial", 9, [[100, 120], [130, 132]]],
                ["full", 11, 13]]},
    {"name": "both partial: intersect with their seq haves",
     "our": {"head": 10, "need": [[2, 5], [7, 7]], "partials": {"9": [[100, 120], [130, 132]]}},
     "their": {"head": 13, "need": [], "partials": {"9": [[100, 110], [130, 130]]}},
     "expect": [["full", 2, 5], ["full", 7, 7], ["partial", 9, [[111, 120], [131, 132]]],
                ["full", 11, 13]]},
]

# agent.rs:1605-1868: sequences of insert_db(set) -> expected gaps; "reset" starts a new
# BookedVersions; final max checked by expect_gaps (agent.rs:1911-1915)
GAPS = [
    {"insert": [[1, 20]], "gaps": []},
    {"insert": [[1, 10]], "gaps": []},
    {"reset": True},
    {"insert": [[1, 1], [4, 4]], "gaps": [[2, 3]]},
    {"insert": [[3, 3], [2, 2]], "gaps": []},
    {"reset": True},
    {"insert": [[5, 20]], "gaps": [[1, 4]]},
    {"insert": [[6, 7]], "gaps": [[1, 4]]},
    {"insert": [[3, 7]], "gaps": [[1, 2]]},
    {"insert": [[1, 2]], "gaps": []},
    {"insert": [[25, 25]], "gaps": [[21, 24]]},
    {"insert": [[30, 35]], "gaps": [[21, 24], [26, 29]]},
    {"insert": [[19, 22]], "gaps": [[23, 24], [26, 29]]},
    {"insert": [[24, 25]], "gaps": [[23, 23], [26, 29]]},
    {"insert": [[23, 27]], "gaps": [[28, 29]]},
    {"insert": [[1, 20]], "gaps": [[28, 29]]},
    {"insert": [[27, 30]], "gaps": []},
    {"insert": [[40, 45]], "gaps": None},
    {"insert": [[50, 55]], "gaps": None},
    {"insert": [[38, 47]], "gaps": [[36, 37], [48, 49]]},
]


# (seqs of the input changes, start_seq, last_seq, max_buf_size in multiples of one change's size
#  or an absolute byte count, expected chunks as (seqs of changes, start, end))
CHUNKER = [
    {"name": "empty iterator", "input": [], "start": 0, "last": 100, "max_bytes": 50,
     "chunks": [[[], 0, 100]]},
    {"name": "2 iterations", "input": [0, 1, 2], "start": 0, "last": 100, "max_changes": 2,
     "chunks": [[[0, 1], 0, 1], [[2], 2, 100]]},
    {"name": "last seq reached", "input": [0, 1], "start": 0, "last": 0, "max_changes": 1,
     "chunks": [[[0], 0, 0]]},
    {"name": "gaps", "input": [0, 2], "start": 0, "last": 100, "max_changes": 2,
     "chunks": [[[0, 2], 0, 100]]},
    {"name": "gaps, send all", "input": [2, 4, 7, 8], "start": 0, "last": 100, "max_bytes": 100000,
     "chunks": [[[2, 4, 7, 8], 0, 100]]},
    {"name": "gaps, two chunks", "input": [2, 4, 7, 8], "start": 0, "last": 10, "max_changes": 2,
     "chunks": [[[2, 4], 0, 4], [[7, 8], 5, 10]]},
]


def _hn_changes():
    """test_handle_need's changes (peer/mod.rs:1757-1781, :1908-1918, :2040-2050, :2076-2108)."""
    c1 = ["tests", 1, "text", T("one"), 1, 1, 0, 1]
    c2 = ["tests", 2, "text", T("two"), 1, 2, 0, 1]
    c3 = ["tests", 1, "text", T("one override"), 2, 3, 0, 1]
    c4 = ["tests", 2, "text", T("two override"), 2, 4, 0, 1]
    wide, seq = [], 0
    for i in range(10):
        grp = []
        pk = {"pack": [i.to_bytes(8, "big").hex(), {"text": str(i)}]}
        vals = [("int", I((i * 7919 - 31337) * 104729)), ("float", R(i * 0.125 - 0.5)),
                ("blob", B(bytes((i * 37 + k * 11) % 256 for k in range(16)).hex()))]
        for col, v in vals:
            grp.append(["wide", pk, col, v, 1, 5, seq, 1])
            seq += 1
        wide.append(grp)
    return c1, c2, c3, c4, wide


def agent_kats():
    ta2 = "11" * 16   # the serving agent's actor (ta2's site id in the reference test)
    bad = "0000000000000000a716446655440000"  # Uuid 00000000-0000-0000-a716-446655440000
    failed = {
        "source": "corro-agent/src/agent/tests.rs:877-999",
        "ta2": ta2, "bad_actor": bad,
        # ta2's five INSERT OR REPLACE INTO tests (id, text) VALUES (i, 'service-text') versions
        "good": [{"actor": ta2, "version": i, "changes": [["tests", i, "text", T("service-text"), 1, i, 0, 1]],
                  "seqs": [0, 0], "last_seq": 0} for i in range(1, 6)],
        "bad": {"actor": bad, "version": 1, "seqs": [0, 1], "last_seq": 1,
                "changes": [["tests", 6, "text", T("six"), 1, 6, 0, 1], ["tests", 6, "nonexistent", T("six"), 1, 6, 1, 1]]},
        # :970-992: crsql_changes db_version of pk i with site_id = ta2 is i; :994-998: no row 6
        "expect_dbv": {str(i): i for i in range(1, 6)}, "expect_absent": [6],
    }
    c1, c2, c3, c4, wide = _hn_changes()
    last = 29

    def full(v, ch, seqs, last_seq=0):
        return {"kind": "full", "version": v, "changes": ch, "seqs": seqs, "last_seq": last_seq}
    flat = [c for g in wide for c in g]
    steps = [
        {"process": [full(1, [c1], [0, 0]), full(2, [c2], [0, 0])]},
        {"need": {"full": [1, 1]}, "expect": [full(1, [c1], [0, 0])]},
        {"need": {"partial": 2, "seqs": [[0, 0]]}, "expect": [full(2, [c2], [0, 0])]},
        {"process": [full(3, [c3], [0, 0])]},
        {"need": {"partial": 1, "seqs": [[0, 0]]}, "expect": [{"kind": "empty", "versions": [1, 1]}]},
        {"need": {"full": [1, 6]}, "expect_prefix": [full(3, [c3], [0, 0]), full(2, [c2], [0, 0]),
                                                     {"kind": "empty", "versions": [1, 1]}]},
        {"process": [full(4, [c4], [0, 0])]},
        {"process": [full(5, g, [g[0][6], g[-1][6]], last) for g in wide]},
        {"need": {"full": [1, 1000]}, "expect_prefix": [full(4, [c4], [0, 0]), full(3, [c3], [0, 0]),
                                                        full(5, flat, [0, last], last),
                                                        {"kind": "empty", "versions": [1, 2]}]},
        {"need": {"partial": 5, "seqs": [[4, 7]]}, "expect": [full(5, flat[4:8], [4, 7], last)]},
        {"need": {"partial": 5, "seqs": [[2, 2], [15, 24]]},
         "expect": [full(5, flat[2:3], [2, 2], last), full(5, flat[15:25], [15, 24], last)]},
    ]
    handle = {"source": "corro-agent/src/api/peer/mod.rs:1729-2321", "actor": "ab" * 16, "ts": 7, "steps": steps}
    return {"process_failed_changes": failed, "handle_need": handle, "clear_empty_versions": clear_empty_versions()}


def clear_empty_versions():
    """test_clear_empty_versions (corro-agent/src/agent/tests.rs:777-875). ta1 writes rows 1..50 of
    tests3, one INSERT OR REPLACE transaction each (insert_rows, tests.rs:1326-1349: text
    'service-name', text2 'second text', num i + 20, num2 i + 100), so version i holds row i's four
    column changes (seqs 0..=3, the range check_bookie_versions asks contains_all for, :1207); then it
    overwrites rows 1..=5, 10, 23..=25, 30..=31 in that order, versions 51..=61 (the same INSERT OR
    REPLACE on an existing row: every column clock bumped to col_version 2). ta2 processes versions
    1..=50 in one process_multiple_changes call and 51..=60 in a second (get_rows, :813-829: version
    61 is not sent); check_bookie_versions then asserts 1..=50 complete (not in gaps); a sync from
    ta2 to ta1 (parallel_sync over generate_sync, :841-849) brings what ta2 needs, and the second
    check asserts that crsql_changes holds no row of site ta1 at versions 1..=5, 10, 23..=25, 30..=31
    (:855-867)."""
    rows = list(range(1, 51))
    over = [1, 2, 3, 4, 5, 10, 23, 24, 25, 30, 31]

    def version(v, row, cv):
        vals = [T("service-name"), T("second text"), I(row + 20), I(row + 100)]
        return {"kind": "full", "version": v, "seqs": [0, 3], "last_seq": 3,
                "changes": [["tests3", row, col, val, cv, v, seq, 1]
                            for seq, (col, val) in enumerate(zip(["text", "text2", "num", "num2"], vals))]}
    ta1_versions = [version(i, r, 1) for i, r in enumerate(rows, 1)] + \
                   [version(51 + k, r, 2) for k, r in enumerate(over)]
    return {"source": "corro-agent/src/agent/tests.rs:777-875 (helpers :1184-1262, :1264-1349)",
            "ta1": "c1" * 16, "ta2": "c2" * 16, "ts": 11,
            "ta1_versions": ta1_versions,
            "calls": [[1, 50], [51, 60]],
            "after_calls": {"complete": [[1, 50]], "gaps": [], "partials": [], "last": 60},
            "sync_needs": [["full", 61, 61]],
            "cleared": [[1, 5], [10, 10], [23, 25], [30, 31]]}


def main():
    merge = [{"name": n, "changes": c, "rows": r, "impacted": imp} for (n, c, r, imp) in MERGE]
    with open(os.path.join(HERE, "merge_kats.json"), "w") as f:
        json.dump({"source": "SURVEY.md App. A.5 + doc/crdts.md:166-245", "cases": merge,
                   "db_versions_case": DBV}, f, indent=1)
    with open(os.path.join(HERE, "sync_kats.json"), "w") as f:
        json.dump({"source": "corro-types/src/sync.rs:386-500", "cases": SYNC}, f, indent=1)
    with open(os.path.join(HERE, "gaps_kats.json"), "w") as f:
        json.dump({"source": "corro-types/src/agent.rs:1605-1868", "steps": GAPS}, f, indent=1)
    with open(os.path.join(HERE, "chunker_kats.json"), "w") as f:
        json.dump({"source": "corro-types/src/change.rs:266-401", "cases": CHUNKER}, f, indent=1)
    with open(os.path.join(HERE, "agent_kats.json"), "w") as f:
        json.dump(agent_kats(), f, indent=1)


if __name__ == "__main__":
    main()
