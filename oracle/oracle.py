"""ctypes binding for liboracle.so — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module, and only
as the checker (or the timed CPU baseline). The product (corrosion_amd) never touches it.
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

OF_INTEGER, OF_REAL, OF_TEXT, OF_BLOB, OF_NULL = 1, 2, 3, 4, 5
OF_LONG = 255  # val_len of a TEXT/BLOB value longer than 16 bytes (bytes in val_data)

_u64p = C.POINTER(C.c_uint64)


class _Changes(C.Structure):
    _fields_ = [("n", C.c_uint64), ("pk", C.c_void_p), ("table_cid", C.c_void_p),
                ("col_version", C.c_void_p), ("db_version", C.c_void_p), ("cl", C.c_void_p),
                ("seq", C.c_void_p), ("site", C.c_void_p), ("val0", C.c_void_p),
                ("val1", C.c_void_p), ("val_type", C.c_void_p), ("val_len", C.c_void_p),
                ("ts", C.c_void_p), ("val_off", C.c_void_p), ("val_size", C.c_void_p),
                ("val_data", C.c_void_p)]


class _Rows(C.Structure):
    _fields_ = [(k, C.c_void_p) for k in ("pk", "table_cid", "col_version", "db_version", "cl",
                                          "seq", "site", "ts", "val0", "val1", "val_type",
                                          "val_len")]


class _SyncEntries(C.Structure):
    _fields_ = [("n", C.c_uint64)] + [(k, C.c_void_p) for k in (
        "their_head", "our_head", "tn_off", "tn_start", "tn_end", "tp_off", "tp_ver", "tps_off",
        "tps_start", "tps_end", "on_off", "on_start", "on_end", "op_off", "op_ver", "ops_off",
        "ops_start", "ops_end")]


class _NeedsOut(C.Structure):
    _fields_ = [(k, C.c_void_p) for k in ("need_count", "seq_count", "need_off", "seq_off", "kind",
                                          "start", "end", "sr_off", "sr_n", "s_start", "s_end")]


_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.of_new.restype = C.c_void_p
        L.of_new.argtypes = [C.c_void_p, C.c_uint32]
        L.of_free.argtypes = [C.c_void_p]
        L.of_apply.argtypes = [C.c_void_p, C.POINTER(_Changes), C.c_void_p]
        L.of_count.restype = C.c_uint64
        L.of_count.argtypes = [C.c_void_p]
        L.of_export.restype = C.c_uint64
        L.of_export.argtypes = [C.c_void_p, C.POINTER(_Rows)]
        L.of_db_versions.argtypes = [C.c_void_p, C.c_void_p]
        L.of_apply_sharded.restype = C.c_int
        L.of_apply_sharded.argtypes = [C.c_void_p, C.c_uint32, C.POINTER(_Changes), C.c_void_p, C.c_uint32]
        L.of_state_digest.argtypes = [C.c_void_p, C.c_void_p]
        L.of_rows_digest.argtypes = [C.POINTER(_Rows), C.c_uint64, C.c_void_p]
        L.of_value_bytes.restype = C.c_uint64
        L.of_value_bytes.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64]
        L.of_bytes_hash.restype = C.c_uint64
        L.of_bytes_hash.argtypes = [C.c_char_p, C.c_uint64]
        L.of_needs.argtypes = [C.POINTER(_SyncEntries), C.POINTER(_NeedsOut), C.c_int]
        L.of_affinity.restype = C.c_int
        L.of_affinity.argtypes = [C.c_int, C.c_int, C.c_uint64, C.c_char_p, C.c_uint64, C.POINTER(C.c_int),
                                  C.POINTER(C.c_uint64), C.c_char_p, C.POINTER(C.c_uint32)]
        L.of_set_affinity.argtypes = [C.c_void_p, C.c_uint32, C.c_char_p, C.c_uint32]
        L.of_booked_new.restype = C.c_void_p
        L.of_booked_free.argtypes = [C.c_void_p]
        L.of_booked_insert_db.restype = C.c_int
        L.of_booked_insert_db.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64]
        L.of_booked_needed_len.restype = C.c_uint64
        L.of_booked_needed_len.argtypes = [C.c_void_p]
        L.of_booked_needed.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        L.of_booked_max.restype = C.c_int64
        L.of_booked_max.argtypes = [C.c_void_p]
        L.of_booked_contains.restype = C.c_int
        L.of_booked_contains.argtypes = [C.c_void_p, C.c_uint64]
        _lib = L
    return _lib


BATCH_DTYPES = {"pk": np.uint64, "table_cid": np.uint32, "col_version": np.int64,
                "db_version": np.int64, "cl": np.uint32, "seq": np.uint32, "site": np.uint32,
                "val0": np.uint64, "val1": np.uint64, "val_type": np.uint8, "val_len": np.uint8,
                "ts": np.uint64, "val_off": np.uint64, "val_size": np.uint32}


def _ptr(a):
    return None if a is None else a.ctypes.data


def _changes_struct(batch, keep):
    n = len(batch["pk"])
    s = _Changes()
    s.n = n
    for k, dt in BATCH_DTYPES.items():
        a = batch.get(k)
        if a is not None:
            a = np.ascontiguousarray(a, dtype=dt)
            assert len(a) == n, k
            keep.append(a)
        setattr(s, k, _ptr(a))
    data = batch.get("val_data")
    if data is not None:
        data = np.frombuffer(bytes(data) or b"\0", np.uint8) if not isinstance(data, np.ndarray) else data
        keep.append(data)
        s.val_data = data.ctypes.data
    return s


def bytes_hash(b):
    """of_bytes_hash: the content hash a long value enters the digests with."""
    b = bytes(b)
    return int(lib().of_bytes_hash(b, len(b)))


class Fold:
    """Sequential cr-sqlite merge fold (crsql_changes INSERT per change)."""

    def __init__(self, site_ids):
        site_ids = np.ascontiguousarray(site_ids, dtype=np.uint8).reshape(-1, 16)
        self._sites = site_ids
        self.nsites = site_ids.shape[0]
        self._h = lib().of_new(site_ids.ctypes.data, self.nsites)

    def __del__(self):
        if getattr(self, "_h", None):
            lib().of_free(self._h)
            self._h = None

    def apply(self, batch):
        keep = []
        s = _changes_struct(batch, keep)
        imp = np.zeros(max(s.n, 1), dtype=np.uint8)
        lib().of_apply(self._h, C.byref(s), imp.ctypes.data)
        return imp[: s.n]

    def set_affinity(self, table, codes):
        """column affinities of `table` (CORRO_AFF_* per cid 1..): winning values are stored converted"""
        b = bytes(bytearray(codes))
        lib().of_set_affinity(self._h, table, b, len(b))

    def export(self):
        return _export_handle(self._h)

    def value_bytes(self, handle):
        return _value_bytes(self._h, handle)

    def db_versions(self):
        out = np.zeros(max(self.nsites, 1), np.int64)
        lib().of_db_versions(self._h, out.ctypes.data)
        return out[: self.nsites]


def _value_bytes(h, handle):
    n = lib().of_value_bytes(h, handle, None, 0)
    buf = C.create_string_buffer(max(n, 1))
    lib().of_value_bytes(h, handle, buf, n)
    return buf.raw[:n]


def _export_handle(h):
    """crsql_changes rows of one fold state (the layout MergeEngine.export() returns)"""
    m = lib().of_count(h)
    out = {"pk": np.zeros(m, np.uint64), "table_cid": np.zeros(m, np.uint32),
           "col_version": np.zeros(m, np.int64), "db_version": np.zeros(m, np.int64),
           "cl": np.zeros(m, np.int64), "seq": np.zeros(m, np.uint32),
           "site": np.zeros(m, np.uint32), "ts": np.zeros(m, np.uint64),
           "val0": np.zeros(m, np.uint64), "val1": np.zeros(m, np.uint64),
           "val_type": np.zeros(m, np.uint8), "val_len": np.zeros(m, np.uint8)}
    r = _Rows()
    for k, a in out.items():
        setattr(r, k, a.ctypes.data if m else None)
    if m:
        got = lib().of_export(h, C.byref(r))
        assert got == m
    out["long_values"] = {int(i): _value_bytes(h, int(out["val1"][i]))
                          for i in np.nonzero(out["val_len"] == OF_LONG)[0]}
    return out


ROW_KEYS = ("table_cid", "pk")  # a clock row's identity (cid is in table_cid's low half)
ROW_VALUE_FIELDS = ("col_version", "db_version", "cl", "seq", "site", "ts", "val0", "val1", "val_type", "val_len")


def rows_diff(got, ref, limit=5):
    """Row-by-row comparison of two crsql_changes exports (MergeEngine.export() / Fold.export() /
    ShardedFold.export()): None when equal, else a report of the row counts and the first `limit`
    differing rows, keyed by (table, cid, pk), so a failed full-size parity check says where. Long
    values compare by their bytes (rows["long_values"]), not by their handles."""
    kdt = np.dtype([("tc", "<u4"), ("pk", "<u8")])

    def keyed(r):
        o = np.lexsort((np.asarray(r["pk"]), np.asarray(r["table_cid"])))
        k = np.empty(len(o), kdt)
        k["tc"] = np.asarray(r["table_cid"])[o]
        k["pk"] = np.asarray(r["pk"])[o]
        return o, k

    def name(k):
        return f"table {int(k['tc']) >> 16} cid {int(k['tc']) & 0xFFFF} pk {int(k['pk'])}"

    og, kg = keyed(got)
    orf, kr = keyed(ref)
    if len(og) != len(orf) or not np.array_equal(kg, kr):
        lines = [f"row sets differ: got {len(og)} rows, expected {len(orf)}"]
        lines += [f"  extra row ({name(k)})" for k in np.setdiff1d(kg, kr)[:limit]]
        lines += [f"  missing row ({name(k)})" for k in np.setdiff1d(kr, kg)[:limit]]
        return "\n".join(lines)
    lg, lr = got.get("long_values") or {}, ref.get("long_values") or {}
    bad = np.zeros(len(og), bool)
    for f in ROW_VALUE_FIELDS:
        a, b = np.asarray(got[f])[og], np.asarray(ref[f])[orf]
        if f == "val1" and (lg or lr):  # long values: handles differ between stores, bytes must not
            is_long = np.asarray(got["val_len"])[og] == OF_LONG
            d = (a != b) & ~is_long
            for j in np.nonzero(is_long)[0]:
                d[j] = lg.get(int(og[j])) != lr.get(int(orf[j]))
            bad |= d
        else:
            bad |= a != b
    idx = np.nonzero(bad)[0]
    if not len(idx):
        return None
    lines = [f"{len(idx)} of {len(og)} rows differ; the first {min(limit, len(idx))}:"]
    for j in idx[:limit]:
        g = {f: int(np.asarray(got[f])[og[j]]) for f in ROW_VALUE_FIELDS}
        r = {f: int(np.asarray(ref[f])[orf[j]]) for f in ROW_VALUE_FIELDS}
        lines.append(f"  {name(kg[j])}: (got, expected) " + str({f: (g[f], r[f]) for f in ROW_VALUE_FIELDS if g[f] != r[f]}))
    return "\n".join(lines)


class ShardedFold:
    """The same fold over `nshards` pk-hash shards with `nthreads` threads (of_apply_sharded):
    rows merge independently, so results equal Fold's. Used as the multi-core CPU baseline and as
    the checker at >= 512M changes (compared through digests)."""

    def __init__(self, site_ids, nshards=16, nthreads=16):
        site_ids = np.ascontiguousarray(site_ids, dtype=np.uint8).reshape(-1, 16)
        self.nsites = site_ids.shape[0]
        self.nthreads = nthreads
        self._hs = (C.c_void_p * nshards)(*[lib().of_new(site_ids.ctypes.data, self.nsites) for _ in range(nshards)])
        self.nshards = nshards

    def __del__(self):
        if getattr(self, "_hs", None) is not None:
            for h in self._hs:
                lib().of_free(h)
            self._hs = None

    def apply(self, batch, impact=True):
        keep = []
        s = _changes_struct(batch, keep)
        imp = np.zeros(max(s.n, 1), dtype=np.uint8) if impact else None
        rc = lib().of_apply_sharded(self._hs, self.nshards, C.byref(s), imp.ctypes.data if impact else None,
                                    self.nthreads)
        assert rc == 0, "batch too large for the sharded fold"
        return imp[: s.n] if impact else None

    def digest(self):
        out = np.zeros(3, np.uint64)
        for h in self._hs:
            lib().of_state_digest(h, out.ctypes.data)
        return tuple(int(x) for x in out)

    def export(self):
        """every shard's rows, concatenated (long-value indices re-based)"""
        parts = [_export_handle(h) for h in self._hs]
        out = {k: np.concatenate([p[k] for p in parts]) for k in parts[0] if k != "long_values"}
        out["long_values"], base = {}, 0
        for p in parts:
            out["long_values"].update({i + base: v for i, v in p["long_values"].items()})
            base += len(p["pk"])
        return out

    def db_versions(self):
        acc = np.full(max(self.nsites, 1), -1, np.int64)
        out = np.zeros(max(self.nsites, 1), np.int64)
        for h in self._hs:
            lib().of_db_versions(h, out.ctypes.data)
            np.maximum(acc, out, out=acc)
        return acc[: self.nsites]


def rows_digest(rows):
    """Digest of crsql_changes rows given as arrays (e.g. MergeEngine.export()), comparable with
    ShardedFold.digest(): (rows, sum of row hashes, xor of rotated row hashes). Rows holding a long
    value (val_len == OF_LONG) need its bytes in rows["long_values"] ({row index: bytes})."""
    m = len(rows["pk"])
    longs = rows.get("long_values") or {}
    if longs:
        rows = dict(rows)
        rows["val1"] = np.array(rows["val1"], dtype=np.uint64, copy=True)
        for i, b in longs.items():
            rows["val1"][i] = bytes_hash(b)
    dts = {"pk": np.uint64, "table_cid": np.uint32, "col_version": np.int64, "db_version": np.int64,
           "cl": np.int64, "seq": np.uint32, "site": np.uint32, "ts": np.uint64, "val0": np.uint64,
           "val1": np.uint64, "val_type": np.uint8, "val_len": np.uint8}
    r = _Rows()
    keep = []
    for k, dt in dts.items():
        a = np.ascontiguousarray(rows[k], dtype=dt)
        keep.append(a)
        setattr(r, k, a.ctypes.data if m else None)
    out = np.zeros(3, np.uint64)
    lib().of_rows_digest(C.byref(r), m, out.ctypes.data)
    return tuple(int(x) for x in out)


SYNC_KEYS_U64 = ("their_head", "tn_off", "tn_start", "tn_end", "tp_off", "tp_ver", "tps_off",
                 "tps_start", "tps_end", "on_off", "on_start", "on_end", "op_off", "op_ver",
                 "ops_off", "ops_start", "ops_end")


def needs(entries):
    """compute_available_needs over CSR entries (dict of numpy arrays). Returns CSR result dict."""
    keep = []
    s = _SyncEntries()
    n = len(entries["their_head"])
    s.n = n
    for k in SYNC_KEYS_U64:
        a = np.ascontiguousarray(entries[k], dtype=np.uint64)
        keep.append(a)
        setattr(s, k, a.ctypes.data if a.size else None)
    oh = np.ascontiguousarray(entries["our_head"], dtype=np.int64)
    keep.append(oh)
    s.our_head = oh.ctypes.data if oh.size else None
    nc = np.zeros(max(n, 1), np.uint64)
    sc = np.zeros(max(n, 1), np.uint64)
    o = _NeedsOut()
    o.need_count = nc.ctypes.data
    o.seq_count = sc.ctypes.data
    lib().of_needs(C.byref(s), C.byref(o), 0)
    nc, sc = nc[:n], sc[:n]
    need_off = np.zeros(n + 1, np.uint64)
    seq_off = np.zeros(n + 1, np.uint64)
    need_off[1:] = np.cumsum(nc)
    seq_off[1:] = np.cumsum(sc)
    T, Ts = int(need_off[-1]), int(seq_off[-1])
    res = {"need_off": need_off, "seq_off": seq_off,
           "kind": np.zeros(max(T, 1), np.uint8), "start": np.zeros(max(T, 1), np.uint64),
           "end": np.zeros(max(T, 1), np.uint64), "sr_off": np.zeros(max(T, 1), np.uint64),
           "sr_n": np.zeros(max(T, 1), np.uint64), "s_start": np.zeros(max(Ts, 1), np.uint64),
           "s_end": np.zeros(max(Ts, 1), np.uint64)}
    for k in ("need_off", "seq_off", "kind", "start", "end", "sr_off", "sr_n", "s_start", "s_end"):
        setattr(o, k, res[k].ctypes.data)
    lib().of_needs(C.byref(s), C.byref(o), 1)
    for k in ("kind", "start", "end", "sr_off", "sr_n"):
        res[k] = res[k][:T]
    for k in ("s_start", "s_end"):
        res[k] = res[k][:Ts]
    return res


def needs_parallel(entries, nthreads=16, chunk=1 << 20):
    """needs() over entry chunks on `nthreads` host threads (the C fold releases the GIL): the CSR
    offsets stay absolute, so a chunk is the per-entry arrays offset by its first entry."""
    from concurrent.futures import ThreadPoolExecutor
    n = len(entries["their_head"])
    keep = {k: np.ascontiguousarray(entries[k], dtype=np.uint64) for k in SYNC_KEYS_U64}
    keep["our_head"] = np.ascontiguousarray(entries["our_head"], dtype=np.int64)
    per_entry = ("their_head", "our_head", "tn_off", "tp_off", "on_off", "op_off")
    nc = np.zeros(max(n, 1), np.uint64)
    sc = np.zeros(max(n, 1), np.uint64)

    def run(a, b, fill, res=None):
        s = _SyncEntries()
        s.n = b - a
        for k in SYNC_KEYS_U64 + ("our_head",):
            arr = keep[k]
            off = a * arr.itemsize if k in per_entry else 0
            setattr(s, k, arr.ctypes.data + off if arr.size else None)
        o = _NeedsOut()
        o.need_count = nc.ctypes.data + 8 * a
        o.seq_count = sc.ctypes.data + 8 * a
        if fill:
            for k in ("kind", "start", "end", "sr_off", "sr_n", "s_start", "s_end"):
                setattr(o, k, res[k].ctypes.data)
            o.need_off = res["need_off"].ctypes.data + 8 * a
            o.seq_off = res["seq_off"].ctypes.data + 8 * a
        lib().of_needs(C.byref(s), C.byref(o), 1 if fill else 0)

    spans = [(a, min(n, a + chunk)) for a in range(0, n, chunk)]
    with ThreadPoolExecutor(nthreads) as ex:
        list(ex.map(lambda ab: run(ab[0], ab[1], False), spans))
    nc, sc = nc[:n], sc[:n]
    need_off = np.zeros(n + 1, np.uint64)
    seq_off = np.zeros(n + 1, np.uint64)
    need_off[1:] = np.cumsum(nc)
    seq_off[1:] = np.cumsum(sc)
    T, Ts = int(need_off[-1]), int(seq_off[-1])
    res = {"need_off": need_off, "seq_off": seq_off,
           "kind": np.zeros(max(T, 1), np.uint8), "start": np.zeros(max(T, 1), np.uint64),
           "end": np.zeros(max(T, 1), np.uint64), "sr_off": np.zeros(max(T, 1), np.uint64),
           "sr_n": np.zeros(max(T, 1), np.uint64), "s_start": np.zeros(max(Ts, 1), np.uint64),
           "s_end": np.zeros(max(Ts, 1), np.uint64)}
    with ThreadPoolExecutor(nthreads) as ex:
        list(ex.map(lambda ab: run(ab[0], ab[1], True, res), spans))
    for k in ("kind", "start", "end", "sr_off", "sr_n"):
        res[k] = res[k][:T]
    for k in ("s_start", "s_end"):
        res[k] = res[k][:Ts]
    return res


class Booked:
    """BookedVersions gap bookkeeping (agent.rs:1108-1235, :1353-1362)."""

    def __init__(self):
        self._h = lib().of_booked_new()

    def __del__(self):
        if getattr(self, "_h", None):
            lib().of_booked_free(self._h)
            self._h = None

    def insert_db(self, ranges):
        s = np.array([r[0] for r in ranges], np.uint64)
        e = np.array([r[1] for r in ranges], np.uint64)
        return lib().of_booked_insert_db(self._h, s.ctypes.data, e.ctypes.data, len(ranges))

    def needed(self):
        m = lib().of_booked_needed_len(self._h)
        s = np.zeros(max(m, 1), np.uint64)
        e = np.zeros(max(m, 1), np.uint64)
        lib().of_booked_needed(self._h, s.ctypes.data, e.ctypes.data)
        return [(int(s[i]), int(e[i])) for i in range(m)]

    def max(self):
        v = lib().of_booked_max(self._h)
        return None if v < 0 else int(v)

    def contains(self, v):
        return bool(lib().of_booked_contains(self._h, v))


def extract_changes(rows, needs):
    """Changeset extraction on exported crsql_changes rows (numpy restatement of handle_need's two
    queries, corro-agent/src/api/peer/mod.rs:385-394 and :423-431 / :603-611): per need, the
    versions of `site` in [start, end] present in the rows, DESCENDING, each with MAX(seq) and
    MAX(ts) over the version's rows and its rows with seq in the optional [seq_start, seq_end],
    by seq ascending (ties by (table_cid, pk), the canonical form the tests compare in). Returns a
    list per need of (version, last_seq, ts, row index array)."""
    site = np.asarray(rows["site"]).astype(np.int64)
    dbv = np.asarray(rows["db_version"]).astype(np.int64)
    order = np.lexsort((np.asarray(rows["pk"]), np.asarray(rows["table_cid"]), np.asarray(rows["seq"]), dbv, site))
    ks, kd = site[order], dbv[order]
    out = []
    for e in range(len(needs["site"])):
        a, s0, e0 = int(needs["site"][e]), int(needs["start"][e]), int(needs["end"][e])
        lo = np.searchsorted(ks, a, "left")
        hi = np.searchsorted(ks, a, "right")
        sub = order[lo:hi]
        d = kd[lo:hi]
        l2, h2 = np.searchsorted(d, s0, "left"), np.searchsorted(d, e0, "right")
        sub, d = sub[l2:h2], d[l2:h2]
        groups = []
        for v in sorted(set(d.tolist()), reverse=True):
            g = sub[d == v]
            last = int(np.asarray(rows["seq"])[g].max())
            ts = int(np.asarray(rows["ts"])[g].max())
            if needs.get("seq_start") is not None:
                sq = np.asarray(rows["seq"])[g]
                g = g[(sq >= int(needs["seq_start"][e])) & (sq <= int(needs["seq_end"][e]))]
            groups.append((v, last, ts, g))
        out.append(groups)
    return out


AFF = {"BLOB": 0, "TEXT": 1, "NUMERIC": 2, "INTEGER": 3, "REAL": 4}


def affinity(aff, value):
    """The value (Python int / float / str / bytes / None) a column of affinity `aff` (AFF code) stores
    for `value` (affinity.c, SQLite 3.37.2 applyAffinity)."""
    import struct
    if value is None or isinstance(value, (bytes, bytearray)):
        return value
    txt = b""
    if isinstance(value, bool) or isinstance(value, int):
        ty, v0 = OF_INTEGER, value & 0xFFFFFFFFFFFFFFFF
    elif isinstance(value, float):
        ty, v0 = OF_REAL, struct.unpack("<Q", struct.pack("<d", value))[0]
    else:
        ty, v0, txt = OF_TEXT, 0, value.encode()
    ot, ov0, olen = C.c_int(), C.c_uint64(), C.c_uint32()
    buf = C.create_string_buffer(32)
    if not lib().of_affinity(aff, ty, v0, txt, len(txt), C.byref(ot), C.byref(ov0), buf, C.byref(olen)):
        return value
    if ot.value == OF_INTEGER:
        return ov0.value - (1 << 64) if ov0.value >> 63 else ov0.value
    if ot.value == OF_REAL:
        return struct.unpack("<d", struct.pack("<Q", ov0.value))[0]
    return buf.raw[: olen.value].decode()
