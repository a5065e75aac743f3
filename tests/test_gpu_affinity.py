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


def _engine(nsites=2, policy="sqlite-3.37.2"):
    """the fixtures pin SQLite 3.37.2's conversions: those tests ask for that policy explicitly"""
    sites = synth.site_ids(nsites, 3)
    e = ca.MergeEngine(SCHEMA, capacity_hint=1 << 16)
    e.register_sites(sites)
    e.set_column_types("t", TYPES)
    e.set_affinity_policy(policy)
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


# ---- the default policy never refuses; the portable policy (opt-in, strict) ----------
def test_default_policy_converts_version_sensitive_values_and_counts_them():
    """A REAL whose '%!.15g' text is another double (0.1 + 0.2) written into a TEXT column applies under
    the default policy -- SQLite stores a converted value and never refuses a change -- and is counted
    in the aff_sensitive metric; a plain conversion is not counted."""
    sites = synth.site_ids(2, 3)
    e = ca.MergeEngine(SCHEMA, capacity_hint=1 << 16)
    e.register_sites(sites)
    e.set_column_types("t", TYPES)
    f = O.Fold(sites)
    f.set_affinity(0, AFF_OF_CID)
    b = _batch([(1, 3, 0.1 + 0.2), (2, 3, 0.5), (3, 1, "12"), (4, 3, 1 / 3)])
    assert np.array_equal(e.apply(b, impact=True), f.apply(b))
    got = _stored(e.export())
    assert got[(1, 3)] == "0.3" and got[(2, 3)] == "0.5" and got[(3, 1)] == 12
    assert sorted(rows_to_tuples(e.export())) == sorted(rows_to_tuples(f.export()))
    assert e.metrics()["aff_sensitive"] == 2



def _sqlite_15g(x):
    """SQLite's "%!.15g" from a correctly rounded '%.15g' (Python's): '.0' when no point, exponent
    with at least two digits (Python's already has them)"""
    s = "%.15g" % x
    m, _, ex = s.partition("e")
    if "." not in m and m not in ("inf", "-inf"):
        m += ".0"
    return m + ("e" + ex if ex else "")


def _correct(aff, v):
    """the value a correctly rounded SQLite stores for v under affinity aff (the conversions the
    portable policy performs), or the marker None when v stays as it is"""
    if aff == "BLOB":
        return None
    if aff == "TEXT":
        if isinstance(v, bool) or not isinstance(v, (int, float)):
            return None
        return str(v) if isinstance(v, int) else _sqlite_15g(v)
    if isinstance(v, str):
        import re
        if not re.fullmatch(r"\s*[+-]?(\d+\.?\d*|\.\d+)([eE][+-]?\d+)?\s*", v):
            return None  # not a number to SQLite (Python's float() also takes 'inf', '1_0', ...)
        r = float(v.strip())
        t = v.strip().lstrip("+-")
        if t.isdigit() and -(1 << 63) <= int(v) < (1 << 63):
            r = int(v)
        elif r.is_integer() and -(2.0 ** 63) < r < 2.0 ** 63:
            r = int(r)
    elif isinstance(v, float):
        r = int(v) if v.is_integer() and -(2.0 ** 63) < v < 2.0 ** 63 else v
    elif isinstance(v, int):
        r = v
    else:
        return None
    if aff == "REAL" and isinstance(r, int):
        r = float(r)
    return r


def _real_text_sensitive(v):
    """a REAL whose '%!.15g' text may differ between SQLite versions: -0.0, infinities, magnitudes
    past 1e307 or below 1e-307 (their text re-reads through the scaled path), or a 15-digit text
    that is another double"""
    return str(v) in ("-0.0", "inf", "-inf") or (v != 0 and not 1e-307 < abs(v) < 1e307) or \
        float(_sqlite_15g(v)) != v


def _text_real_sensitive(v):
    """a decimal text whose double may differ between SQLite versions: more than 15 significant
    digits, an extreme magnitude, or an exact value within 2^-50 (relative) of a double rounding midpoint"""
    import math
    from fractions import Fraction
    t = v.strip()
    mant = t.lstrip("+-").lower().split("e")[0].replace(".", "").lstrip("0").rstrip("0")
    if len(mant) > 15:
        return True
    x = Fraction(t)
    if x == 0:
        return False
    try:
        d = float(x)
    except OverflowError:
        return True
    if math.isinf(d) or abs(d) < 2.2250738585072014e-308 or abs(d) > 1e300:
        return True
    nb = math.nextafter(d, math.inf if Fraction(d) < x else -math.inf)
    mid = (Fraction(d) + Fraction(nb)) / 2
    return abs(x - mid) / abs(x) < Fraction(1, 1 << 50)


def _one(e, cid, v):
    """apply one change; the stored value, or the string 'refused'"""
    e.reset()
    try:
        e.apply(_batch([(1, cid, v)]))
    except ca.CorroError as err:
        assert err.code == -6 and "SQLite version" in str(err)
        return "refused"
    return _stored(e.export()).get((1, cid))


def test_portable_policy_converts_only_version_independent_values():
    """Every fixture case under the portable policy: either refused as a whole batch (CORRO_E_RANGE,
    nothing written), or stored exactly as SQLite 3.37.2 stores it (the fixture) AND as a correctly
    rounded conversion stores it (Python's float() / '%.15g'). A refusal is only allowed where the
    15-digit rendering does not round-trip (REAL -> TEXT) or the decimal needs more than 15 digits or
    an extreme exponent (TEXT -> REAL)."""
    d = json.load(open(os.path.join(HERE, "golden", "affinity_kats.json")))
    e, _ = _engine(policy="portable")
    refused = converted = 0
    for c in d["cases"]:
        aff, v, want = c["affinity"], _decode(c["in"]), _decode(c["out"])
        got = _one(e, CID_OF_AFF[aff], v)
        if got == "refused":
            refused += 1
            if aff == "TEXT":
                assert isinstance(v, float) and _real_text_sensitive(v), (aff, v)
            else:
                assert isinstance(v, str) and _text_real_sensitive(v), (aff, v)
            continue
        converted += 1
        assert _key(got) == _key(want), (aff, v, got, want)
        cr = _correct(aff, v)
        if cr is not None:
            assert _key(got) == _key(cr), (aff, v, got, cr)
    assert converted > 450 and refused > 0


@pytest.mark.parametrize("aff,v,refuse", [
    ("TEXT", 0.1 + 0.2, True),             # '%!.15g' -> '0.3', which is another double
    ("TEXT", 0.5, False),
    ("TEXT", -0.0, True),                  # 3.37.2 writes '0.0'
    ("TEXT", -2.25, False),
    ("TEXT", 1e20, False),                 # '1.0e+20'
    ("TEXT", 1 / 3, True),
    ("REAL", "0.1000000000000000055511151231257827021181583404541015625", True),  # dropped digits
    ("REAL", "1e400", True),               # overflow
    ("REAL", "4.9e-324", True),            # subnormal
    ("REAL", "2.5", False),
    ("NUMERIC", " 12.0 ", False),          # INTEGER 12
    ("INTEGER", "9007199254740993", False),  # integer text: exact
    ("REAL", "9007199254740993", False),   # int64 -> double: correctly rounded in every version
    ("NUMERIC", "9007199254740993.0", False),  # an integer after the '.0' is stripped: (double)s
    ("REAL", "1.000000000000000111", True),  # 19 digits, within the long double's margin of 1 + 2^-53
])
def test_portable_policy_known_cases(aff, v, refuse):
    e, _ = _engine(policy="portable")
    got = _one(e, CID_OF_AFF[aff], v)
    assert (got == "refused") == refuse, (aff, v, got)
    if not refuse:
        cr = _correct(aff, v)
        assert _key(got) == _key(cr), (aff, v, got, cr)
    e37, _ = _engine()
    assert _one(e37, CID_OF_AFF[aff], v) != "refused"


def test_portable_refusal_writes_nothing():
    e, _ = _engine(policy="portable")
    e.apply(_batch([(1, 1, 5)]))
    before = sorted(rows_to_tuples(e.export()))
    with pytest.raises(ca.CorroError):
        e.apply(_batch([(2, 2, 7), (3, 3, 0.1 + 0.2)]))
    assert sorted(rows_to_tuples(e.export())) == before
