"""Primary keys beyond one INTEGER column: every table of corro-tests' TEST_SCHEMA
(/root/reference/crates/corro-tests/src/lib.rs:13-53) -- tests, tests2, tests3 (INTEGER pk),
testsblob (BLOB pk), testsbool, wide (composite BLOB + TEXT pk) -- merged through the C ABI with
interned row keys (corro_pk_keys) and checked against the oracle on the same keys, bit-exact; the
keys map back to the canonical packed pks (corro_pk_bytes)."""
import numpy as np
import pytest

import synth
from oracle import oracle as O
from tests._util import rows_to_tuples

pytestmark = pytest.mark.gpu

SCHEMA = {"tests": ["text"], "tests2": ["text"], "tests3": ["text", "text2", "num", "num2"],
          "testsblob": ["text"], "testsbool": ["b"], "wide": ["int", "float", "blob"]}
INTERNED = ("testsblob", "wide")


def _pack(cols):
    """pack_columns (pubsub.rs:2304-2358) of ints / bytes (BLOB) / str (TEXT)."""
    from corrosion_amd.serve import num_bytes_needed_i64
    out = bytes([len(cols)])

    def nb32(v):
        return 4 if v & 0xFF000000 else 3 if v & 0xFF0000 else 2 if v & 0xFF00 else 1 if v else 0
    for c in cols:
        if isinstance(c, int):
            n = num_bytes_needed_i64(c)
            out += bytes([(n << 3) | 1]) + (c & ((1 << (8 * n)) - 1)).to_bytes(n, "big") if n else bytes([1])
        else:
            b = c.encode() if isinstance(c, str) else bytes(c)
            n = nb32(len(b))
            out += bytes([(n << 3) | (3 if isinstance(c, str) else 4)]) + len(b).to_bytes(n, "big") + b
    return out


def _changes(rng, n, nsites):
    tables = list(SCHEMA)
    rows = []
    for i in range(n):
        t = tables[int(rng.integers(0, len(tables)))]
        k = int(rng.integers(0, 60))
        if t == "testsblob":
            pk = _pack([bytes([k, k * 7 % 256]) * (1 + k % 5)])
        elif t == "wide":
            pk = _pack([k.to_bytes(8, "big"), str(k % 7)])
        else:
            pk = _pack([k - 10])
        cols = SCHEMA[t]
        sent = rng.random() < 0.15
        cid = 0 if sent else int(rng.integers(1, len(cols) + 1))
        cl = int(rng.integers(1, 5))
        cl = cl if sent else (cl | 1)
        cv = cl if sent else int(rng.integers(1, 4))
        if sent:
            vt, v0, v1, vl = 5, 0, 0, 0
        else:
            col = cols[cid - 1]
            if col in ("num", "num2", "int", "b"):
                vt, v0, v1, vl = 1, int(rng.integers(0, 4)), 0, 0
            elif col == "float":
                vt, v0, v1, vl = 2, int(np.float64(rng.integers(0, 3) * 0.5).view(np.uint64)), 0, 0
            elif col == "blob":
                raw = bytes(rng.integers(0, 3, 16, dtype=np.uint8))
                vt, v0, v1, vl = 4, int.from_bytes(raw[:8], "big"), int.from_bytes(raw[8:], "big"), 16
            else:
                s = f"v{int(rng.integers(0, 3))}".encode()
                vt, v0, v1, vl = 3, int.from_bytes(s.ljust(8, b"\0"), "big"), 0, len(s)
        rows.append((t, pk, cid, vt, v0, v1, vl, cv, int(rng.integers(1, 50)), int(rng.integers(0, nsites)), cl, i))
    return rows


def test_every_corro_tests_table_vs_oracle():
    import corrosion_amd as ca
    rng = np.random.default_rng(3)
    sites = synth.site_ids(6, 3)
    e = ca.MergeEngine(SCHEMA, capacity_hint=1 << 14, interned=INTERNED)
    e.register_sites(sites)
    f = O.Fold(sites)
    tix = {t: i for i, t in enumerate(SCHEMA)}
    for batch_no in range(3):
        rows = _changes(rng, 6000, len(sites))
        keys = np.zeros(len(rows), np.uint64)
        for t in SCHEMA:
            idx = [j for j, r in enumerate(rows) if r[0] == t]
            if not idx:
                continue
            if t in INTERNED:
                keys[idx] = e.pk_keys(t, [rows[j][1] for j in idx])
            else:
                from corrosion_amd.wire import unpack_int_pk
                keys[idx] = [unpack_int_pk(rows[j][1]) & 0xFFFFFFFFFFFFFFFF for j in idx]
        b = {"pk": keys,
             "table_cid": np.array([(tix[r[0]] << 16) | r[2] for r in rows], np.uint32),
             "val_type": np.array([r[3] for r in rows], np.uint8),
             "val0": np.array([r[4] for r in rows], np.uint64),
             "val1": np.array([r[5] for r in rows], np.uint64),
             "val_len": np.array([r[6] for r in rows], np.uint8),
             "col_version": np.array([r[7] for r in rows], np.int64),
             "db_version": np.array([r[8] for r in rows], np.int64),
             "site": np.array([r[9] for r in rows], np.uint32),
             "cl": np.array([r[10] for r in rows], np.uint32),
             "seq": np.array([r[11] % 100 for r in rows], np.uint32)}
        assert np.array_equal(e.apply(b, impact=True), f.apply(b))
        assert rows_to_tuples(e.export()) == rows_to_tuples(f.export())
    # interned keys give back the canonical packed pks, every table's rows present
    got = e.export()
    for t in INTERNED:
        m = (got["table_cid"] >> 16) == tix[t]
        assert m.any()
        for k, pk in zip(got["pk"][m][:50], e.pk_bytes(t, got["pk"][m][:50])):
            assert e.pk_keys(t, [pk])[0] == k
    e.close()


def test_noncanonical_pk_encodings_name_one_row():
    """A non-canonical packed integer (more bytes than needed) inside a composite key is the same
    row as the canonical one (cr-sqlite re-packs pks)."""
    import corrosion_amd as ca
    e = ca.MergeEngine(SCHEMA, capacity_hint=1 << 12, interned=INTERNED)
    canon = _pack([b"\x00" * 7 + b"\x05", "5"])
    longer = bytes([2, (1 << 3) | 4, 8]) + b"\x00" * 7 + b"\x05" + bytes([(4 << 3) | 3]) + (1).to_bytes(4, "big") + b"5"
    k1, k2 = e.pk_keys("wide", [canon, longer])
    assert k1 == k2
    assert e.pk_bytes("wide", [k1])[0] == canon
    with pytest.raises(ca.CorroError):
        e.pk_keys("tests", [canon])  # a composite pk on a single-INTEGER-pk table
    e.close()
