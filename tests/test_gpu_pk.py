"""Primary keys beyond one INTEGER column: every table of corro-tests' TEST_SCHEMA
(/root/reference/crates/corro-tests/src/lib.rs:13-53) -- tests, tests2, tests3 (INTEGER pk),
testsblob (BLOB pk), testsbool, wide (composite BLOB + TEXT pk) -- merged through the C ABI with
interned row keys (corro_pk_keys) and checked against the oracle on the same keys, bit-exact; the
keys map back to the canonical packed pks (corro_pk_bytes). TEXT / BLOB column values have any
length (SqliteValue, corro-api-types/src/lib.rs:419-429): values longer than 16 bytes go through
the value arena and compare by their whole bytes."""
import numpy as np
import pytest

import synth
from oracle import oracle as O
from tests._util import encode_values, rows_to_tuples

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
            val = None
        else:
            col = cols[cid - 1]
            if col in ("num", "num2", "int", "b"):
                val = int(rng.integers(0, 4))
            elif col == "float":
                val = float(rng.integers(0, 3) * 0.5)
            elif col == "blob":
                val = BLOBS[int(rng.integers(0, len(BLOBS)))]
            else:
                val = TEXTS[int(rng.integers(0, len(TEXTS)))]
        rows.append((t, pk, cid, val, cv, int(rng.integers(1, 50)), int(rng.integers(0, nsites)), cl, i))
    return rows


# short and long values that tie on their first 8 / 16 bytes, differ only past them, or only in length
TEXTS = ["v0", "v1", "v2", "hello world, this is a long text value", "hello world, this is a long text valuf",
         "hello world, this is a long text value!", "hello wo", "0123456789abcdef", "0123456789abcdef0",
         "0123456789abcdef" * 20]
BLOBS = [bytes(16), bytes(17), bytes(16) + b"\1", bytes([1, 2]) * 20, bytes([1, 2]) * 21, bytes([1, 2, 2]) * 7,
         bytes(range(3)) * 5 + bytes([9])]


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
             "col_version": np.array([r[4] for r in rows], np.int64),
             "db_version": np.array([r[5] for r in rows], np.int64),
             "site": np.array([r[6] for r in rows], np.uint32),
             "cl": np.array([r[7] for r in rows], np.uint32),
             "seq": np.array([r[8] % 100 for r in rows], np.uint32)}
        b.update(encode_values([r[3] for r in rows]))
        assert "val_data" in b
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
