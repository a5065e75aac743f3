"""Test helpers: turn golden-fixture notation into SoA batches (numpy) and back."""
import json
import os
import struct

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
TYPES = {"int": 1, "real": 2, "text": 3, "blob": 4, "null": 5}


def load_golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def site_table(n=16):
    """sN = sixteen bytes of value N (SURVEY A.5 notation); ordinal N."""
    return np.array([[i] * 16 for i in range(n)], dtype=np.uint8)


def encode_value(v):
    t = TYPES[v["t"]]
    if t == 1:
        return t, int(v["v"]) & 0xFFFFFFFFFFFFFFFF, 0, 0
    if t == 2:
        return t, struct.unpack("<Q", struct.pack("<d", float(v["v"])))[0], 0, 0
    if t in (3, 4):
        b = v["v"].encode() if t == 3 else bytes.fromhex(v["v"])
        assert len(b) <= 16
        p = b + b"\0" * (16 - len(b))
        return t, int.from_bytes(p[:8], "big"), int.from_bytes(p[8:], "big"), len(b)
    return 5, 0, 0, 0


def batch_from_changes(changes, pk=1, table=0, seq0=0):
    """changes: [cid, value, cv, dbv, site, cl] rows -> SoA dict"""
    n = len(changes)
    b = {k: [] for k in ("pk", "table_cid", "col_version", "db_version", "cl", "seq", "site",
                         "val0", "val1", "val_type", "val_len", "ts")}
    for i, (cid, val, cv, dbv, site, cl) in enumerate(changes):
        t, v0, v1, ln = encode_value(val)
        b["pk"].append(pk)
        b["table_cid"].append((table << 16) | cid)
        b["col_version"].append(cv)
        b["db_version"].append(dbv)
        b["cl"].append(cl)
        b["seq"].append(seq0 + i)
        b["site"].append(site)
        b["val0"].append(v0)
        b["val1"].append(v1)
        b["val_type"].append(t)
        b["val_len"].append(ln)
        b["ts"].append(1000 + dbv)
    dt = {"pk": np.uint64, "table_cid": np.uint32, "col_version": np.int64, "db_version": np.int64,
          "cl": np.uint32, "seq": np.uint32, "site": np.uint32, "val0": np.uint64,
          "val1": np.uint64, "val_type": np.uint8, "val_len": np.uint8, "ts": np.uint64}
    return {k: np.array(v, dtype=dt[k]) for k, v in b.items()}


LONG = 255  # val_len of a TEXT/BLOB value longer than 16 bytes


def encode_values(vals):
    """SqliteValues (None | int | float | str | bytes, any length) -> the batch's value fields:
    val_type / val0 / val1 / val_len, plus val_off / val_size / val_data for values longer than 16
    bytes (omitted when there are none)."""
    n = len(vals)
    out = {"val_type": np.zeros(n, np.uint8), "val0": np.zeros(n, np.uint64), "val1": np.zeros(n, np.uint64),
           "val_len": np.zeros(n, np.uint8)}
    off, size, data, dlen = np.zeros(n, np.uint64), np.zeros(n, np.uint32), [], 0
    for i, v in enumerate(vals):
        if v is None:
            out["val_type"][i] = 5
        elif isinstance(v, (bool, int)):
            out["val_type"][i], out["val0"][i] = 1, int(v) & 0xFFFFFFFFFFFFFFFF
        elif isinstance(v, float):
            out["val_type"][i], out["val0"][i] = 2, struct.unpack("<Q", struct.pack("<d", v))[0]
        else:
            b = v.encode() if isinstance(v, str) else bytes(v)
            out["val_type"][i] = 3 if isinstance(v, str) else 4
            if len(b) > 16:
                out["val0"][i], out["val_len"][i] = int.from_bytes(b[:8], "big"), LONG
                off[i], size[i] = dlen, len(b)
                data.append(b)
                dlen += len(b)
            else:
                p = b.ljust(16, b"\0")
                out["val0"][i], out["val1"][i] = int.from_bytes(p[:8], "big"), int.from_bytes(p[8:], "big")
                out["val_len"][i] = len(b)
    if data:
        out["val_off"], out["val_size"] = off, size
        out["val_data"] = np.frombuffer(b"".join(data), np.uint8)
    return out


def rows_to_tuples(rows, with_ts=False):
    """exported state dict -> sorted list of comparable tuples (a long value compares by its bytes,
    rows["long_values"])"""
    n = len(rows["pk"])
    longs = rows.get("long_values") or {}
    out = []
    for i in range(n):
        t = int(rows["val_type"][i])
        lv = t in (3, 4) and int(rows["val_len"][i]) == LONG
        tup = (int(rows["table_cid"][i]) >> 16, int(rows["pk"][i]), int(rows["table_cid"][i]) & 0xFFFF,
               t, int(rows["val0"][i]) if t != 5 else 0,
               (longs[i] if lv else int(rows["val1"][i])) if t in (3, 4) else 0,
               int(rows["val_len"][i]) if t in (3, 4) else 0, int(rows["col_version"][i]),
               int(rows["db_version"][i]), int(rows["site"][i]), int(rows["cl"][i]),
               int(rows["seq"][i]))
        if with_ts:
            tup = tup + (int(rows["ts"][i]),)
        out.append(tup)
    out.sort()
    return out


def expected_rows(rows, pk=1, table=0):
    out = []
    for (cid, val, cv, dbv, site, cl) in rows:
        t, v0, v1, ln = encode_value(val)
        out.append((table, pk, cid, t, v0 if t != 5 else 0, v1 if t in (3, 4) else 0,
                    ln if t in (3, 4) else 0, cv, dbv, site, cl))
    out.sort()
    return out
