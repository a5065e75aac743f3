"""The oracle's restatement of SQLite column affinity (oracle/affinity.c) against SQLite itself: the
committed fixtures (tests/golden/affinity_kats.json, stdlib sqlite3 3.37.2) and live comparisons with
the stdlib sqlite3 on random integers, doubles and numeric texts. (SQLite is not the reference: it is
the library the reference's cr-sqlite runs inside, and its conversion decides what the base table
holds after a change wins)"""
import json
import os
import random
import sqlite3
import struct

import pytest

from oracle import oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
AFFS = ["TEXT", "NUMERIC", "INTEGER", "REAL", "BLOB"]


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


def _key(v):
    """type and exact value (REAL by bits: -0.0 != 0.0)"""
    if isinstance(v, float):
        return ("REAL", struct.pack("<d", v))
    return (type(v).__name__, v)


def test_fixtures():
    d = json.load(open(os.path.join(HERE, "golden", "affinity_kats.json")))
    assert d["cases"]
    for c in d["cases"]:
        got = O.affinity(O.AFF[c["affinity"]], _decode(c["in"]))
        assert _key(got) == _key(_decode(c["out"])), c


def _sqlite_store(values):
    con = sqlite3.connect(":memory:")
    con.execute("CREATE TABLE t (id INTEGER PRIMARY KEY, " + ", ".join(f"c{k} {a}" for k, a in enumerate(AFFS)) + ")")
    con.executemany("INSERT INTO t VALUES (?, ?, ?, ?, ?, ?)", [(i,) + (v,) * 5 for i, v in enumerate(values)])
    return con.execute("SELECT c0, c1, c2, c3, c4 FROM t ORDER BY id").fetchall()


def _random_values(rng, n):
    out = []
    for _ in range(n):
        k = rng.randrange(7)
        if k == 0:
            out.append(rng.randrange(-(1 << 63), 1 << 63) >> rng.randrange(64))
        elif k == 1:  # any finite double
            while True:
                x = struct.unpack("<d", struct.pack("<Q", rng.getrandbits(64)))[0]
                if x == x and abs(x) != float("inf"):
                    break
            out.append(x)
        elif k == 2:  # doubles near decimal boundaries
            out.append(rng.choice([1, -1]) * rng.randrange(1, 10 ** 17) * 10.0 ** rng.randrange(-30, 30))
        elif k == 3:  # integral doubles
            out.append(float(rng.randrange(-(1 << 62), 1 << 62) >> rng.randrange(62)))
        else:  # numeric-looking text
            sp = lambda: rng.choice(["", "", " ", "\t", "  "])
            digits = "".join(rng.choice("0123456789") for _ in range(rng.randrange(0, 25)))
            frac = "." + "".join(rng.choice("0123456789") for _ in range(rng.randrange(0, 20))) \
                if rng.random() < 0.6 else ""
            exp = (rng.choice("eE") + rng.choice(["", "+", "-"]) + str(rng.randrange(0, 400))) \
                if rng.random() < 0.4 else ""
            junk = rng.choice(["", "", "", "", "x", "e", "1e", "."])
            out.append(sp() + rng.choice(["", "", "-", "+"]) + digits + frac + exp + junk + sp())
    return out


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_random_values_match_sqlite(seed):
    rng = random.Random(seed)
    vals = _random_values(rng, 6000)
    rows = _sqlite_store(vals)
    bad = []
    for v, row in zip(vals, rows):
        for a, got in zip(AFFS, row):
            mine = O.affinity(O.AFF[a], v)
            if _key(mine) != _key(got):
                bad.append((a, v, got, mine))
    assert not bad, bad[:10]
