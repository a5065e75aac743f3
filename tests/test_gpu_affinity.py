"""Column affinity: a winning value is stored as its column's affinity converts it
(SQLite 3.37.2's conversion, emulated on the device including its x87 long-double decimal scaling),
and the next incoming change is compared unconverted against that stored value. Checked against
the committed SQLite fixtures and against the oracle (oracle/affinity.c, itself pinned against the
stdlib sqlite3 by tests/test_affinity_oracle.py) on random values, through every merge path."""
import json
import os
import random
import struct
import sys

import numpy as np
import pytest

import corrosion_amd as ca
import synth
from oracle import oracle as O
from tests._util import encode_values, rows_to_tuples

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
I, R, T, B, N = 1, 2, 3, 4, 5
SCHEMA = {"t": ["i", "r", "s", "b", "n"]}
TYPES = ["INTEGER", "REAL", "TEXT", "BLOB", "NUMERIC"]   # cid 1..5
AFF_OF_CID = [O.AFF["INTEGER"], O.AFF["REAL"], O.AFF["TEXT"], O.AFF["BLOB"], O.AFF["NUMERIC"]]
CID_OF_AFF = {"INTEGER": 1, "REAL": 2, "TEXT": 3, "BLOB": 4, "NUMERIC": 5}


def _batch(rows, cv=None, site=None):
    """rows: (pk, cid, value) -> a batch with cl 1, col_version 1 (or cv), site 0 (or site)"""
    n = len(rows)
    out = {"pk": np.array([r[0] for r in rows], np.uint64), "table_cid": np.array([r[1] for r in rows], np.uint32),
           "col_version": np.ones(n, np.int64) if cv is None else np.asarray(cv, np.int64),
           "db_version": np.arange(1, n + 1, dtype=np.int64),
           "cl": np.ones(n, np.uint32), "seq": np.zeros(n, np.uint32),
           "site": np.zeros(n, np.uint32) if site is None else np.asarray(site, np.uint32)}
    out.update(encode_values([r[2] for r in rows]))
    return out


def _engine(nsites=2):
    sites = synth.site_ids(nsites, 3)
    e = ca.MergeEngine(SCHEMA, capacity_hint=1 << 16)
    e.register_sites(sites)
    e.set_column_types("t", TYPES)
    f = O.Fold(sites)
    f.set_affinity(0, AFF_OF_CID)
    return e, f


def _stored(rows):
    """{(pk, cid): python value} of an export"""
    out = {}
    longs = rows.get("long_values") or {}
    for k in range(len(rows["pk"])):
        cid = int(rows["table_cid"][k]) & 0xFFFF
        if cid == 0:
            continue
        t, v0, v1, ln = (int(rows["val_type"][k]), int(rows["val0"][k]), int(rows["val1"][k]),
                         int(rows["val_len"][k]))
        if t == I:
            v = v0 - (1 << 64) if v0 >> 63 else v0
        elif t == R:
            v = struct.unpack("<d", struct.pack("<Q", v0))[0]
        elif t in (T, B):
            raw = longs[k] if ln == 255 else (v0.to_bytes(8, "big") + v1.to_bytes(8, "big"))[:ln]
            v = raw.decode() if t == T else bytes(raw)
        else:
            v = None
        out[(int(rows["pk"][k]), cid)] = v
    return out


def _key(v):
    return ("REAL", struct.pack("<d", v)) if isinstance(v, float) else (type(v).__name__, v)


def _decode(e):
    t = e["type"]
    if t == "INTEGER":
        return int(e["int"])
    if t == "REAL":
        return struct.unpack("<d", struct.pack("<Q", int(e["bits"], 16)))[0]
    if t == "TEXT":
        return bytes.fromhex(e["hex"]).decode()
    if t == "BLOB":
        return bytes.fromhex(e["hex"])
    return None


def test_values_in_their_class_merge_exactly():
    e, f = _engine()
    rows = [(1, 1, 5), (1, 2, 5.5), (1, 3, "abc"), (1, 4, b"\x00\x01"), (1, 5, 2.5),
            (2, 1, "not a number"), (2, 2, "x1"), (2, 3, b"12"), (2, 4, 7), (2, 5, 9),
            (3, 1, 5.5), (3, 4, 1.0), (3, 5, "1e"), (3, 3, None)]
    b = _batch(rows)
    imp = e.apply(b, impact=True)
    assert np.array_equal(imp, f.apply(b))
    assert sorted(rows_to_tuples(e.export())) == sorted(rows_to_tuples(f.export()))


def test_pinned_conversions_match_sqlite_fixtures():
    """every (value, affinity) case of tests/golden/affinity_kats.json (stdlib sqlite3 3.37.2),
    the App. A.4 probes among them: int 5 -> TEXT '5', -0.0 -> INTEGER 0, int 5 -> REAL 5.0"""
    d = json.load(open(os.path.join(HERE, "golden", "affinity_kats.json")))
    rows, want = [], {}
    for k, c in enumerate(d["cases"]):
        cid = CID_OF_AFF[c["affinity"]]
        rows.append((k, cid, _decode(c["in"])))
        want[(k, cid)] = _decode(c["out"])
    e, f = _engine()
    e.apply(_batch(rows))
    got = _stored(e.export())
    bad = [(k, rows[k[0]][2], got[k], w) for k, w in want.items() if _key(got[k]) != _key(w)]
    assert not bad, bad[:10]
    probes = {(5, 3): "5", (-0.0, 1): 0, (5, 2): 5.0}
    for (v, cid), w in probes.items():
        k = next(i for i, r in enumerate(rows) if r[1] == cid and _key(r[2]) == _key(v))
        assert _key(got[(k, cid)]) == _key(w)


def _random_values(seed, n):
    sys.path.insert(0, HERE)
    from test_affinity_oracle import _random_values as rv
    vals = rv(random.Random(seed), n)
    rng = random.Random(seed + 1)
    for k in range(0, n, 37):  # long texts: numeric with padding, and not numeric
        vals[k] = " " * rng.randrange(1, 12) + str(rng.randrange(-(10 ** 25), 10 ** 25)) + " " * rng.randrange(0, 9) \
            if k % 2 else "x" * rng.randrange(17, 40)
    for k in range(5, n, 101):
        vals[k] = rng.choice([None, b"12", b"\x00" * 20, float("inf"), -float("inf")])
    return vals


@pytest.mark.parametrize("seed", [11, 12])
def test_random_values_every_affinity_vs_oracle(seed):
    vals = _random_values(seed, 20000)
    rows = [(k, 1 + (k * 7 + seed) % 5, v) for k, v in enumerate(vals)]
    e, f = _engine()
    b = _batch(rows)
    imp = e.apply(b, impact=True)
    assert np.array_equal(imp, f.apply(b))
    got, want = _stored(e.export()), _stored(f.export())
    bad = [(k, vals[k[0]], got[k], want[k]) for k in want if _key(got[k]) != _key(want[k])]
    assert not bad, bad[:10]
    assert sorted(rows_to_tuples(e.export())) == sorted(rows_to_tuples(f.export()))


@pytest.mark.parametrize("hot", [False, True])
def test_raw_versus_stored_comparison_order(hot):
    """conflicting changes (same col_version) to the same cells mix values the affinity converts: each
    incoming change compares raw against the stored (converted) value, in application order. hot=True
    puts thousands of them on one row (the overflow path's sequential fold)."""
    rng = random.Random(5 + hot)
    pool = [5, "5", 5.0, "5.0", -0.0, 0, "0", 7, "7", "abc", 2.5, "2.5", " 12 ", 12, 12.0, b"5", None, "1e3", 1000]
    n = 60000 if hot else 20000
    npk = 4 if hot else 2000
    rows = [(rng.randrange(npk), 1 + rng.randrange(5), rng.choice(pool)) for _ in range(n)]
    cv = [rng.randrange(1, 3) for _ in range(n)]
    site = [rng.randrange(4) for _ in range(n)]
    e, f = _engine(4)
    b = _batch(rows, cv, site)
    imp = e.apply(b, impact=True)
    assert np.array_equal(imp, f.apply(b))
    assert sorted(rows_to_tuples(e.export())) == sorted(rows_to_tuples(f.export()))
    # a second batch onto the stored state
    rows2 = [(rng.randrange(npk), 1 + rng.randrange(5), rng.choice(pool)) for _ in range(n // 2)]
    b2 = _batch(rows2, [rng.randrange(1, 4) for _ in range(n // 2)], [rng.randrange(4) for _ in range(n // 2)])
    assert np.array_equal(e.apply(b2, impact=True), f.apply(b2))
    assert sorted(rows_to_tuples(e.export())) == sorted(rows_to_tuples(f.export()))


def test_long_numeric_text_converted():
    e, f = _engine()
    txt = "   12345678901234567890   "
    b = _batch([(1, 1, txt), (2, 3, -123456789012345678), (3, 3, -1.2345678901234e-300), (4, 2, txt)])
    e.apply(b)
    f.apply(b)
    got = _stored(e.export())
    assert got[(1, 1)] == 1.2345678901234567e+19 and got[(2, 3)] == "-123456789012345678"
    assert got[(3, 3)] == "-1.2345678901234e-300" and got[(4, 2)] == 1.2345678901234567e+19
    assert sorted(rows_to_tuples(e.export())) == sorted(rows_to_tuples(f.export()))
