"""Fixtures of SQLite column affinity (tests/golden/affinity_kats.json): for each value of a chosen set
and each affinity (TEXT, NUMERIC, INTEGER, REAL, BLOB), the storage class and value SQLite reads back
after an INSERT into a column of that affinity -- what cr-sqlite's base table holds after a change
wins (the column types come from corrosion's schema, corro-types/src/schema.rs:274).

Generated with the Python stdlib sqlite3 module (SQLite 3.37.2 in this image; affinity conversion is
SQLite's own code, not cr-sqlite's). Re-run: python tests/golden/make_affinity.py
"""
import json
import os
import sqlite3
import struct

HERE = os.path.dirname(os.path.abspath(__file__))

AFFS = {"TEXT": "TEXT", "NUMERIC": "NUMERIC", "INTEGER": "INTEGER", "REAL": "REAL", "BLOB": "BLOB"}

INTS = [0, 1, 5, -7, 42, 1 << 31, (1 << 53) - 1, 1 << 53, (1 << 53) + 1, 10 ** 15, 10 ** 16 - 1, 10 ** 16,
        1234567890123456789, (1 << 63) - 1, -(1 << 63)]
REALS = [0.0, -0.0, 5.0, -3.0, 2.5, 0.1, 1e15 - 1, 1e15, 1e16, 123456789.0, -123456789012345.0, 1e300, -1e-300,
         9.2e18, 9.3e18, -9.3e18, 0.5, 1.0 / 3.0, 4503599627370496.0, 9007199254740993.0, float("inf"),
         -float("inf"), 5e-324, 2.2250738585072014e-308, 1.7976931348623157e308, 0.1 + 0.2, 123.456, 1e-5, 1e-4,
         -9223372036854775808.0, 0.000123456789012345678, 99999999999999.99, 999999999999999.9]
TEXTS = ["5", " 12 ", "+7", "-0", "007", "3.0", "3.0e+5", "1e3", "1E2", "1.5", ".5", "5.", "+.5", "-.5e1", "1e",
         "1e+", "abc", "12abc", "0x10", "", " ", "\t42\n", "9223372036854775807", "9223372036854775808",
         "-9223372036854775808", "-9223372036854775809", "1.0", "  -12.000  ", "2.0000000000000000001",
         "123456789012345678", "   12345678901234567890   ", "0.1", "1e308", "1e309", "-0.0", "4.5e15",
         "9007199254740993.0", "9007199254740993", "12345678901234567890123", "1.5e-3", "7e-0", "8E+01",
         "392e296", "76574689900994988418859e+70", "9330591241.28464921439603345e-253", "1e-320", "5e-324",
         "2e-400", "-1e400", "1e341", "123456789012345678901234567890e280", "0.000000000000000000000000001",
         "1.7976931348623157e308", "1.8e308", "+", "-", ".", "e5", "1.2.3", "1e5x", "0x", "   ", "\v7\f"]
BLOBS = [b"", b"5", b"12", b"\x00\x01", b"1.5"]


def encode(v):
    if v is None:
        return {"type": "NULL"}
    if isinstance(v, int):
        return {"type": "INTEGER", "int": str(v)}
    if isinstance(v, float):
        return {"type": "REAL", "bits": "%016x" % struct.unpack("<Q", struct.pack("<d", v))[0]}
    if isinstance(v, str):
        return {"type": "TEXT", "hex": v.encode().hex()}
    return {"type": "BLOB", "hex": bytes(v).hex()}


def main():
    con = sqlite3.connect(":memory:")
    cols = ", ".join(f"c_{a.lower()} {t}" for a, t in AFFS.items())
    con.execute(f"CREATE TABLE t (id INTEGER PRIMARY KEY, {cols})")
    out = {"sqlite_version": sqlite3.sqlite_version, "cases": []}
    vals = INTS + REALS + TEXTS + BLOBS + [None]
    for i, v in enumerate(vals):
        con.execute(f"INSERT INTO t VALUES (?, {', '.join('?' for _ in AFFS)})", [i] + [v] * len(AFFS))
        row = con.execute(f"SELECT {', '.join(f'c_{a.lower()}' for a in AFFS)} FROM t WHERE id = ?", (i,)).fetchone()
        for a, got in zip(AFFS, row):
            out["cases"].append({"affinity": a, "in": encode(v), "out": encode(got)})
    with open(os.path.join(HERE, "affinity_kats.json"), "w") as f:
        json.dump(out, f, indent=0)
    print(len(out["cases"]), "cases,", "sqlite", sqlite3.sqlite_version)


if __name__ == "__main__":
    main()
