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


def rows_to_tuples(rows, with_ts=False):
    """exported state dict -> sorted list of comparable tuples"""
    n = len(rows["pk"])
    out = []
    for i in range(n):
        t = int(rows["val_type"][i])
        tup = (int(rows["table_cid"][i]) >> 16, int(rows["pk"][i]), int(rows["table_cid"][i]) & 0xFFFF,
               t, int(rows["val0"][i]) if t != 5 else 0, int(rows["val1"][i]) if t in (3, 4) else 0,
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
