"""Primary keys beyond one INTEGER column: every table of corro-tests' TEST_SCHEMA
(/root/reference/crates/corro-tests/src/lib.rs:13-53) -- tests, tests2, tests3 (INTEGER pk),
testsblob (BLOB pk), testsbool, wide (composite BLOB + TEXT pk) -- merged through the C ABI with
interned row keys (corro_pk_keys) and checked against the oracle on the same keys, bit-exact; the
keys map back to the canonical packed pks (corro_pk_bytes). TEXT / BLOB column values have any
length (SqliteValue, corro-api-types/src/lib.rs:419-429): values longer than 16 bytes go through
the value arena and compare by their whole bytes."""
import os
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


def _canon(b):
    import ctypes as C
    from corrosion_amd import _lib as L
    out = (C.c_uint8 * (9 * len(b) + 16))()
    n = C.c_uint64()
    L.check(L.lib().corro_pk_canonical(bytes(b), len(b), out, len(out), C.byref(n)))
    return bytes(out[:n.value])


def _noncanonical(rng, b):
    """another encoding of the same key: an INTEGER column's value sign-extended from more bytes, or a
    BLOB / TEXT length written with a wider length prefix (unpack_columns reads both)"""
    ncol, pos, out = b[0], 1, bytearray([b[0]])
    for _c in range(ncol):
        tb = b[pos]
        t, n = tb & 7, tb >> 3
        if t == 1:
            v = int.from_bytes(b[pos + 1:pos + 1 + n], "big", signed=True) if n else 0
            m = min(8, n + 1 + int(rng.integers(0, 2)))
            out += bytes([(m << 3) | 1]) + (v & ((1 << (8 * m)) - 1)).to_bytes(m, "big")
            pos += 1 + n
        elif t in (3, 4):
            ln = int.from_bytes(b[pos + 1:pos + 1 + n], "big") if n else 0
            m = min(4, n + 1)
            out += bytes([(m << 3) | t]) + ln.to_bytes(m, "big") + b[pos + 1 + n:pos + 1 + n + ln]
            pos += 1 + n + ln
        else:
            sz = 8 if t == 2 else 0
            out += b[pos:pos + 1 + sz]
            pos += 1 + sz
    return bytes(out)


@pytest.mark.parametrize("device_api", [False, True])
def test_intern_table_keys_are_a_persistent_bijection(device_api):
    """The HBM intern table (corro_pk_keys stages host pks into it; corro_pk_keys_device takes them
    where they lie): over three calls of random testsblob / wide pks -- duplicates inside a call, keys
    re-sent in later calls, non-canonical encodings -- equal canonical pks get one key, distinct ones
    distinct keys, the keys are dense (0 .. n-1 over the calls) and stable across calls, and every key
    maps back to its canonical bytes (corro_pk_bytes)."""
    import torch
    import corrosion_amd as ca
    rng = np.random.default_rng(5 + device_api)
    e = ca.MergeEngine(SCHEMA, capacity_hint=1 << 12, interned=INTERNED)
    seen = {}
    for call in range(3):
        for table in ("testsblob", "wide"):
            pool = [_pack([bytes(rng.integers(0, 256, int(rng.integers(0, 40)), dtype=np.uint8))]) if table == "testsblob"
                    else _pack([int(rng.integers(-2**40, 2**40)).to_bytes(8, "big", signed=True), str(int(rng.integers(0, 50)))])
                    for _ in range(3000)]
            pks = [pool[int(rng.integers(0, len(pool)))] for _ in range(8000)]
            pks = [_noncanonical(rng, p) if rng.random() < 0.1 else p for p in pks]
            if device_api:
                buf = torch.tensor(list(b"".join(pks)) or [0], dtype=torch.uint8, device="cuda")
                off = torch.tensor(np.concatenate([[0], np.cumsum([len(p) for p in pks])]), dtype=torch.int64,
                                   device="cuda")
                keys = e.pk_keys_device(table, buf, off).cpu().numpy().view(np.uint64)
            else:
                keys = e.pk_keys(table, pks)
            got = seen.setdefault(table, {})
            for p, k in zip(pks, keys.tolist()):
                c = _canon(p)
                assert got.setdefault(c, k) == k, (table, call)
            inv = {}
            for c, k in got.items():
                assert inv.setdefault(k, c) == c
            assert sorted(inv) == list(range(len(inv)))
    for table, got in seen.items():
        ks = np.array(list(got.values()), np.uint64)
        assert e.pk_bytes(table, ks) == list(got.keys())


def test_device_intern_rejects_malformed_pk():
    import torch
    import corrosion_amd as ca
    e = ca.MergeEngine(SCHEMA, capacity_hint=1 << 12, interned=INTERNED)
    good = _pack([b"abc"])
    bad = bytes([1, (5 << 3) | 4, 200, 1, 2])   # a 200-byte BLOB with 2 bytes
    buf = torch.tensor(list(good + bad), dtype=torch.uint8, device="cuda")
    off = torch.tensor([0, len(good), len(good) + len(bad)], dtype=torch.int64, device="cuda")
    with pytest.raises(ca.CorroError):
        e.pk_keys_device("testsblob", buf, off)
    with pytest.raises(ca.CorroError):   # a composite pk on a table keyed by one INTEGER
        e.pk_keys_device("tests", buf[:len(good)], off[:2])


@pytest.mark.slow
def test_blob_pk_config2_size_vs_sharded_oracle():
    """Config 2 at its full size (2^26 changes, 2^22 rows, 1000 actors) over a testsblob-shaped table:
    every pk a 16-byte BLOB packed in HBM (19 bytes), interned on the device (corro_pk_keys_device),
    then applied with impacts. The keys are a bijection of the row ids, stable when the same pks come
    again; impacts, every output row (pk mapped back to its row id) and db_versions equal the oracle's
    pk-sharded fold of the batch keyed by the row ids."""
    import torch
    import corrosion_amd as ca
    sites = synth.site_ids(1000, 1)
    b = synth.uniform_batch_torch(1 << 26, 1000, 1 << 22, 4, seed=synth.config_seed(2), device="cuda")
    ids = b["pk"]
    data, off = synth.blob_pks_torch(ids)
    e = ca.MergeEngine({"t": ["a", "b", "c", "d"]}, capacity_hint=1 << 26, interned=("t",))
    e.register_sites(sites)
    keys = e.pk_keys_device("t", data, off)
    uid, inv = torch.unique(ids, return_inverse=True)
    kmax = torch.full((uid.numel(),), -1, dtype=torch.int64, device="cuda").scatter_reduce(0, inv, keys, "amax")
    kmin = torch.full((uid.numel(),), 1 << 62, dtype=torch.int64, device="cuda").scatter_reduce(0, inv, keys, "amin")
    assert torch.equal(kmax, kmin)                                   # one key per row id
    assert torch.unique(kmax).numel() == uid.numel() == int(kmax.max()) + 1  # distinct, dense
    again = e.pk_keys_device("t", data[:19 * 4096], off[:4097])
    assert torch.equal(again, keys[:4096])                           # stable across calls
    bb = dict(b)
    bb["pk"] = keys
    imp = e.apply(bb, impact=True).cpu().numpy()
    hb = {k: v.cpu().numpy() for k, v in b.items()}
    id_of_key = torch.empty(uid.numel(), dtype=torch.int64, device="cuda")
    id_of_key[kmax] = uid
    del b, bb, data, off, keys, kmax, kmin, inv
    torch.cuda.empty_cache()
    for k in ("table_cid", "cl", "seq", "site"):
        hb[k] = hb[k].view(np.uint32)
    for k in ("pk", "val0"):
        hb[k] = hb[k].view(np.uint64)
    f = O.ShardedFold(sites, nshards=64, nthreads=16)
    ref = f.apply(hb)
    assert np.array_equal(imp, ref)
    rows = e.export()
    rows["pk"] = id_of_key.cpu().numpy().view(np.uint64)[rows["pk"].astype(np.int64)]
    assert O.rows_digest(rows) == f.digest()
    assert np.array_equal(e.db_versions(), f.db_versions())
    e.close()


def test_intern_table_grows_past_its_probe_bound():
    """A call bringing far more new keys than the table was sized for (1.5 M after 1000): probes run
    past PK_MAX_PROBE, the call retries on tables four times larger (rebuilt from the keys on the
    device) until every key finds a slot -- the earlier keys keep their ids, the new ones are dense
    after them, duplicates inside the call share one id, and ids map back to their bytes."""
    import torch
    import corrosion_amd as ca
    import synth
    e = ca.MergeEngine(SCHEMA, capacity_hint=1 << 12, interned=INTERNED)
    ids1 = torch.arange(1000, device="cuda")
    b1, o1 = synth.blob_pks_torch(ids1)
    k1 = e.pk_keys_device("testsblob", b1, o1).cpu().numpy().view(np.uint64)
    assert sorted(k1.tolist()) == list(range(1000))
    n2 = 1_500_000
    ids2 = torch.cat([torch.arange(n2, device="cuda"), torch.arange(0, n2, 7, device="cuda")])  # (with repeats)
    b2, o2 = synth.blob_pks_torch(ids2)
    k2 = e.pk_keys_device("testsblob", b2, o2).cpu().numpy().view(np.uint64)
    assert np.array_equal(k2[:1000], k1)                      # earlier keys keep their ids
    first = k2[:n2]
    assert np.unique(first).size == n2 and int(first.max()) == n2 - 1  # dense, one id per distinct key
    assert np.array_equal(k2[n2:], first[::7])                # repeats inside the call share the id
    rng = np.random.default_rng(3)
    pick = rng.integers(0, n2, 200)
    got = e.pk_bytes("testsblob", first[pick])
    raw = b2.cpu().numpy()
    assert got == [bytes(raw[19 * i:19 * i + 19]) for i in pick.tolist()]


def test_intern_ids_follow_first_seen_order():
    """New keys get ids in first-seen order (cr-sqlite numbers __crsql_key rows in insertion
    order; the device claims are won by whichever change's CAS lands first, so the ids are ranked by
    each key's first change instead): over two calls with repeats, non-canonical encodings and keys
    longer than a slot's inline bytes, a key's id is the table size before the call plus the rank of its
    first occurrence among the call's new keys -- the same on a fresh engine, run after run."""
    import torch
    import corrosion_amd as ca
    rng = np.random.default_rng(11)
    pool = [_pack([bytes(rng.integers(0, 256, int(rng.integers(0, 60)), dtype=np.uint8))]) for _ in range(5000)]
    calls = []
    for _ in range(2):
        pks = [pool[int(rng.integers(0, len(pool)))] for _ in range(20000)]
        calls.append([_noncanonical(rng, p) if rng.random() < 0.1 else p for p in pks])
    want, ids = [], {}
    for pks in calls:
        got = []
        for p in pks:
            c = _canon(p)
            if c not in ids:
                ids[c] = len(ids)
            got.append(ids[c])
        want.append(got)
    for run in range(2):
        e = ca.MergeEngine(SCHEMA, capacity_hint=1 << 12, interned=INTERNED)
        for pks, w in zip(calls, want):
            buf = torch.tensor(list(b"".join(pks)), dtype=torch.uint8, device="cuda")
            off = torch.tensor(np.concatenate([[0], np.cumsum([len(p) for p in pks])]), dtype=torch.int64, device="cuda")
            keys = e.pk_keys_device("testsblob", buf, off).cpu().numpy().view(np.uint64)
            assert keys.tolist() == w, run
        e.close()


@pytest.mark.parametrize("fault", ["pk_find", "pk_commit"])
def test_failed_intern_leaves_the_table_as_it_was(fault):
    """a call that fails after its probe pass has claimed slots (injected: CORRO_FAULT
    pk_find before the probe, pk_commit after it) leaves no claim behind -- a retry of the same batch, and
    a shorter batch whose indices a stale claim would point past, intern exactly as on a fresh table."""
    import torch
    import corrosion_amd as ca
    rng = np.random.default_rng(13)
    e = ca.MergeEngine(SCHEMA, capacity_hint=1 << 12, interned=INTERNED)
    held = torch.arange(500, device="cuda")
    bh, oh = synth.blob_pks_torch(held)
    kh = e.pk_keys_device("testsblob", bh, oh).cpu().numpy().view(np.uint64)
    ids = torch.tensor(rng.integers(0, 3000, 40000), device="cuda")
    b, o = synth.blob_pks_torch(ids)
    os.environ["CORRO_FAULT"] = fault
    try:
        with pytest.raises(ca.CorroError):
            e.pk_keys_device("testsblob", b, o)
    finally:
        del os.environ["CORRO_FAULT"]
    short = synth.blob_pks_torch(ids[:1000])
    ks = e.pk_keys_device("testsblob", *short).cpu().numpy().view(np.uint64)
    k = e.pk_keys_device("testsblob", b, o).cpu().numpy().view(np.uint64)
    f = ca.MergeEngine(SCHEMA, capacity_hint=1 << 12, interned=INTERNED)
    assert np.array_equal(f.pk_keys_device("testsblob", bh, oh).cpu().numpy().view(np.uint64), kh)
    assert np.array_equal(f.pk_keys_device("testsblob", *short).cpu().numpy().view(np.uint64), ks)
    assert np.array_equal(f.pk_keys_device("testsblob", b, o).cpu().numpy().view(np.uint64), k)
    idn = ids.cpu().numpy()
    assert all(k[i] == kh[idn[i]] for i in range(len(idn)) if idn[i] < 500)  # held keys keep their ids
    e.close()
    f.close()


def _rebuild_digest():
    """Keys of three calls on one table: 200 K new keys (a rebuild after the call: a quarter of the table
    new), a call with 600 K more (growth), then every key again (a warm call through the rebuilt table)."""
    import hashlib
    import torch
    import corrosion_amd as ca
    e = ca.MergeEngine(SCHEMA, capacity_hint=1 << 12, interned=INTERNED)
    h = hashlib.sha256()
    for ids in (torch.arange(200_000, device="cuda"), torch.arange(100_000, 800_000, device="cuda"),
                torch.arange(800_000, device="cuda").flip(0)):
        k = e.pk_keys_device("testsblob", *synth.blob_pks_torch(ids)).cpu().numpy().view(np.uint64)
        h.update(k.tobytes())
    e.close()
    return h.hexdigest()


def test_intern_rebuild_in_home_order_matches_rebuild_by_claims():
    """The table rebuilt from the arena in home order (sorted homes, max-scan positions; the default)
    and by claims (CORRO_PK_ORDERED=0, also the fallback when the pad runs out) intern every call to
    the same keys: ids are first-seen ranks whatever the slot layout, and a warm call re-finds every key
    through the rebuilt table."""
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    ordered = _rebuild_digest()
    code = ("import sys; sys.path[:0] = [%r, %r]; import test_gpu_pk as t; print(t._rebuild_digest())" % (root, here))
    env = dict(os.environ, CORRO_PK_ORDERED="0")
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240, cwd=root)
    assert out.returncode == 0, out.stderr[-2000:]
    assert out.stdout.strip().splitlines()[-1] == ordered
