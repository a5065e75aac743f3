"""Column affinity: values already in the class their column's affinity keeps merge
exactly; a value the affinity would convert fails the batch (CORRO_E_RANGE) with the state untouched."""
import struct

import numpy as np
import pytest

import corrosion_amd as ca
import synth
from oracle import oracle as O
from tests._util import rows_to_tuples

pytestmark = pytest.mark.gpu

I, R, T, B, N = 1, 2, 3, 4, 5
SCHEMA = {"t": ["i", "r", "s", "b", "n"]}
TYPES = ["INTEGER", "REAL", "TEXT", "BLOB", "NUMERIC"]   # cid 1..5


def _be(b):
    b = b + bytes(16 - len(b))
    return int.from_bytes(b[:8], "big"), int.from_bytes(b[8:16], "big")


def _batch(rows):
    """rows: (pk, cid, type, value) -> a batch with cl 1, col_version 1, site 0."""
    n = len(rows)
    out = {"pk": np.array([r[0] for r in rows], np.uint64), "table_cid": np.array([r[1] for r in rows], np.uint32),
           "col_version": np.ones(n, np.int64), "db_version": np.arange(1, n + 1, dtype=np.int64),
           "cl": np.ones(n, np.uint32), "seq": np.zeros(n, np.uint32), "site": np.zeros(n, np.uint32),
           "val0": np.zeros(n, np.uint64), "val1": np.zeros(n, np.uint64), "val_type": np.zeros(n, np.uint8),
           "val_len": np.zeros(n, np.uint8)}
    for k, (_pk, _cid, ty, v) in enumerate(rows):
        out["val_type"][k] = ty
        if ty == I:
            out["val0"][k] = np.int64(v).view(np.uint64)
        elif ty == R:
            out["val0"][k] = struct.unpack("<Q", struct.pack("<d", v))[0]
        elif ty in (T, B):
            w0, w1 = _be(v)
            out["val0"][k], out["val1"][k], out["val_len"][k] = w0, w1, len(v)
    return out


def _engine():
    sites = synth.site_ids(2, 3)
    e = ca.MergeEngine(SCHEMA, capacity_hint=4096)
    e.register_sites(sites)
    e.set_column_types("t", TYPES)
    return e, sites


def test_values_in_their_class_merge_exactly():
    e, sites = _engine()
    rows = [(1, 1, I, 5), (1, 2, R, 5.5), (1, 3, T, b"abc"), (1, 4, B, b"\x00\x01"), (1, 5, R, 2.5),
            (2, 1, T, b"not a number"), (2, 2, T, b"x1"), (2, 3, B, b"12"), (2, 4, I, 7), (2, 5, I, 9),
            (3, 1, R, 5.5), (3, 4, R, 1.0), (3, 5, T, b"1e"), (3, 3, N, None)]
    b = _batch(rows)
    imp = e.apply(b, impact=True)
    f = O.Fold(sites)
    assert np.array_equal(imp, f.apply(b))
    assert sorted(rows_to_tuples(e.export())) == sorted(rows_to_tuples(f.export()))


@pytest.mark.parametrize("row", [
    (1, 1, R, 5.0),            # INTEGER column: a REAL holding an integer becomes INTEGER
    (1, 1, R, -0.0),           # ... -0.0 too (stored as int 0, App. A.4 probe)
    (1, 1, T, b" 12 "),        # ... a numeric text becomes a number
    (1, 2, I, 5),              # REAL column: INTEGER becomes REAL
    (1, 2, T, b"-1.5e3"),
    (1, 3, I, 5),              # TEXT column: numbers become text
    (1, 3, R, 0.25),
    (1, 5, R, 3.0),            # NUMERIC column
    (1, 5, T, b"+.5"),
])
def test_values_the_affinity_converts_are_refused(row):
    e, _sites = _engine()
    e.apply(_batch([(9, 1, I, 1)]))
    before = rows_to_tuples(e.export())
    with pytest.raises(ca.CorroError, match="CORRO_E_RANGE"):
        e.apply(_batch([(4, 4, B, b"ok"), row]))
    assert rows_to_tuples(e.export()) == before


def test_long_numeric_text_refused():
    e, _sites = _engine()
    b = _batch([(1, 1, I, 1)])
    txt = b"   12345678901234567890   "
    b["val_type"][0], b["val_len"][0] = T, 255
    b["val_off"] = np.zeros(1, np.uint64)
    b["val_size"] = np.array([len(txt)], np.uint32)
    b["val_data"] = np.frombuffer(txt, np.uint8).copy()
    with pytest.raises(ca.CorroError, match="CORRO_E_RANGE"):
        e.apply(b)
