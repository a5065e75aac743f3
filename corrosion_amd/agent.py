"""Mirror of corrosion's apply entry points over the device engine.

Types mirror corro-types: `Change` (change.rs:19-30), `ChangeV1` / `Changeset::{Full, Empty,
EmptySet}` (broadcast.rs:114-148); functions mirror corro-agent/src/agent/util.rs:
`process_multiple_changes` (:691), `process_fully_buffered_changes` (:541) and corro-types
`generate_sync` (sync.rs:284). All logic runs in libcorro_hip.so (csrc/agent.cpp + the HIP merge);
this module converts the Python objects to the C ABI structs and back.
"""
import ctypes as C
import struct
from dataclasses import dataclass, field

import numpy as np

from . import _lib as L
from .engine import MergeEngine
from .sync import SyncStateV1


@dataclass
class Change:
    table: str
    pk: object              # INTEGER pk value, or pack_columns bytes (interned tables: any pk)
    cid: str                # column name, "-1" = row sentinel
    val: object             # None | int | float | str | bytes  (SqliteValue)
    col_version: int
    db_version: int
    seq: int
    site_id: bytes          # 16 bytes
    cl: int


@dataclass
class Full:
    version: int
    changes: list
    seqs: tuple             # (start, end) inclusive
    last_seq: int
    ts: int = 0


@dataclass
class Empty:
    versions: tuple         # (start, end) inclusive
    ts: int = None


@dataclass
class EmptySet:
    versions: list
    ts: int = 0


@dataclass
class ChangeV1:
    actor_id: bytes
    changeset: object


def value_bytes(v):
    """The bytes of a TEXT/BLOB SqliteValue (None for other classes)."""
    if v is None or isinstance(v, (bool, int, float)):
        return None
    return v.encode() if isinstance(v, str) else bytes(v)


def encode_value(v):
    """SqliteValue -> (type, val0, val1, len) of the engine's fixed-width value encoding. A TEXT/BLOB
    longer than 16 bytes gives len = CORRO_VAL_LONG and its first 8 bytes in val0: its bytes travel in
    the batch's val_data (value_bytes)."""
    if v is None:
        return L_NULL, 0, 0, 0
    if isinstance(v, bool) or isinstance(v, int):
        return 1, int(v) & 0xFFFFFFFFFFFFFFFF, 0, 0
    if isinstance(v, float):
        if v != v:
            return L_NULL, 0, 0, 0  # SQLite binds NaN as NULL
        return 2, struct.unpack("<Q", struct.pack("<d", v))[0], 0, 0
    b = v.encode() if isinstance(v, str) else bytes(v)
    if len(b) > 16:
        if len(b) >= 1 << 24:
            raise L.CorroError(-6, "TEXT/BLOB values of 16 MiB or more are outside the engine encoding")
        return (3 if isinstance(v, str) else 4), int.from_bytes(b[:8], "big"), 0, L.CORRO_VAL_LONG
    p = b + b"\0" * (16 - len(b))
    return (3 if isinstance(v, str) else 4), int.from_bytes(p[:8], "big"), int.from_bytes(p[8:], "big"), len(b)


L_NULL = 5


@dataclass
class Processed:
    known: list                               # per ChangeV1: "skipped" | "current" | "cleared" | "partial" | error code
    impactful: list = field(default_factory=list)  # per ChangeV1: impactful Change list (Full only)
    ready: list = field(default_factory=list)      # (actor, version) now fully buffered


class Bookie:
    def __init__(self):
        h = C.c_void_p()
        L.check(L.lib().corro_bookie_new(C.byref(h)))
        self._h = h

    def __del__(self):
        if getattr(self, "_h", None):
            L.lib().corro_bookie_free(self._h)
            self._h = None

    def last(self, actor):
        v = C.c_int64()
        L.check(L.lib().corro_bookie_last(self._h, actor, C.byref(v)))
        return None if v.value < 0 else v.value

    def needed(self, actor):
        c = C.c_uint64()
        L.check(L.lib().corro_bookie_needed(self._h, actor, None, None, 0, C.byref(c)))
        s = np.zeros(max(1, c.value), np.uint64)
        e = np.zeros(max(1, c.value), np.uint64)
        L.check(L.lib().corro_bookie_needed(self._h, actor, s.ctypes.data, e.ctypes.data, c.value, C.byref(c)))
        return [(int(s[i]), int(e[i])) for i in range(c.value)]

    def contains_all(self, actor, versions, seqs=None):
        r = C.c_int()
        L.check(L.lib().corro_bookie_contains_all(self._h, actor, versions[0], versions[1], 1 if seqs else 0,
                                                   seqs[0] if seqs else 0, seqs[1] if seqs else 0, C.byref(r)))
        return bool(r.value)

    def partial(self, actor, version):
        """(seq ranges, last_seq) of a partially received version, or None."""
        c, last = C.c_uint64(), C.c_int64()
        # sizing call first (cap 0), then the ranges: a version may hold any number of seq ranges
        L.check(L.lib().corro_bookie_partial(self._h, actor, version, None, None, 0, C.byref(c), C.byref(last)))
        if last.value < 0:
            return None
        n = int(c.value)
        s = np.zeros(max(n, 1), np.uint64)
        e = np.zeros(max(n, 1), np.uint64)
        L.check(L.lib().corro_bookie_partial(self._h, actor, version, s.ctypes.data, e.ctypes.data, n,
                                             C.byref(c), C.byref(last)))
        return [(int(s[i]), int(e[i])) for i in range(n)], int(last.value)


class Agent:
    """One node's writer: the device merge engine + its Bookie (agent.rs:480-482 single writer)."""

    def __init__(self, schema, capacity_hint=1 << 20, device=0, actor_id=b"\0" * 16, interned=()):
        self.engine = MergeEngine(schema, capacity_hint=capacity_hint, device=device, interned=interned)
        self.bookie = Bookie()
        self.actor_id = actor_id
        self.site_ids = {}      # ordinal -> 16-byte site id (crsql_site_id)

    def row_keys(self, changes):
        """Row keys of the changes' primary keys: an INTEGER pk is its own key; an interned table's
        pk (pack_columns bytes, or an int packed as one INTEGER column) goes through corro_pk_keys."""
        from .wire import pack_int_pk, unpack_int_pk
        keys = np.zeros(len(changes), np.uint64)
        by_table = {}
        for j, ch in enumerate(changes):
            if ch.table in self.engine.interned:
                packed = bytes(ch.pk) if isinstance(ch.pk, (bytes, bytearray)) else pack_int_pk(ch.pk)
                by_table.setdefault(ch.table, ([], []))
                by_table[ch.table][0].append(j)
                by_table[ch.table][1].append(packed)
            elif isinstance(ch.pk, (bytes, bytearray)):
                keys[j] = unpack_int_pk(bytes(ch.pk)) & 0xFFFFFFFFFFFFFFFF
            else:
                keys[j] = ch.pk & 0xFFFFFFFFFFFFFFFF
        for table, (idx, packed) in by_table.items():
            keys[idx] = self.engine.pk_keys(table, packed)
        return keys

    def site(self, site_id):
        o = int(self.engine.register_sites(np.frombuffer(bytes(site_id), np.uint8).reshape(1, 16))[0])
        self.site_ids[o] = bytes(site_id)
        return o

    def change_queue(self, **kw):
        """handle_changes' batching loop in front of this agent (queue.ChangeQueue): apply each batch
        it returns with process_multiple_changes, then report it with job_done()."""
        from .queue import ChangeQueue
        return ChangeQueue(self.actor_id, self.bookie.contains_all, **kw)

    def handle_needs(self, needs, max_buf_size=None):
        """Answer (actor_id, SyncNeedV1) needs from this node's state (serve.handle_needs)."""
        from . import serve
        return serve.handle_needs(self, needs, max_buf_size or serve.MAX_CHANGES_BYTES_PER_MESSAGE)

    def process_multiple_changes(self, changes):
        """changes: list of ChangeV1 (or (ChangeV1, source, instant) tuples) in arrival order."""
        changes = [c[0] if isinstance(c, tuple) else c for c in changes]
        ncs = len(changes)
        rows = []
        descs = (L.Changeset * max(1, ncs))()
        actor_bufs = []
        for i, cv1 in enumerate(changes):
            cs = cv1.changeset
            d = descs[i]
            ab = C.create_string_buffer(bytes(cv1.actor_id), 16)
            actor_bufs.append(ab)
            d.actor_id = C.addressof(ab)
            d.site = self.site(cv1.actor_id)
            d.change_off = len(rows)
            if isinstance(cs, Full):
                d.kind = L.CORRO_CS_FULL
                d.version_start = d.version_end = cs.version
                d.seq_start, d.seq_end = cs.seqs
                d.last_seq = cs.last_seq
                d.ts = cs.ts or 0
                d.change_count = len(cs.changes)
                rows.extend(cs.changes)
            elif isinstance(cs, Empty):
                d.kind = L.CORRO_CS_EMPTY
                d.version_start, d.version_end = cs.versions
                d.ts = cs.ts or 0
            else:
                d.kind = L.CORRO_CS_EMPTY_SET
                d.ts = cs.ts or 0
        n = len(rows)
        arr = {k: np.zeros(max(1, n), dt) for k, dt in (
            ("pk", np.uint64), ("table_cid", np.uint32), ("col_version", np.int64), ("db_version", np.int64),
            ("cl", np.uint32), ("seq", np.uint32), ("site", np.uint32), ("val0", np.uint64),
            ("val1", np.uint64), ("val_type", np.uint8), ("val_len", np.uint8))}
        arr["pk"][:n] = self.row_keys(rows)
        voff, vsz, data = np.zeros(max(1, n), np.uint64), np.zeros(max(1, n), np.uint32), []
        dlen = 0
        for j, ch in enumerate(rows):
            try:
                tc = self.engine.lookup(ch.table, ch.cid)
            except L.CorroError:
                tc = L.CORRO_TCID_UNKNOWN
            t, v0, v1, ln = encode_value(ch.val)
            arr["table_cid"][j] = tc
            arr["col_version"][j] = ch.col_version
            arr["db_version"][j] = ch.db_version
            arr["cl"][j] = ch.cl
            arr["seq"][j] = ch.seq
            arr["site"][j] = self.site(ch.site_id)
            arr["val0"][j], arr["val1"][j], arr["val_type"][j], arr["val_len"][j] = v0, v1, t, ln
            if ln == L.CORRO_VAL_LONG:
                b = value_bytes(ch.val)
                voff[j], vsz[j] = dlen, len(b)
                data.append(b)
                dlen += len(b)
        s = L.Changes()
        s.n = n
        for k, a in arr.items():
            setattr(s, k, a.ctypes.data)
        s.ts = None
        if data:
            blob = np.frombuffer(b"".join(data), np.uint8)
            s.val_off, s.val_size, s.val_data, s.val_data_len = voff.ctypes.data, vsz.ctypes.data, blob.ctypes.data, dlen
        known = np.zeros(max(1, ncs), np.int32)
        imp = np.zeros(max(1, n), np.uint8)
        out = L.ProcessOut()
        out.known = known.ctypes.data
        out.impactful = imp.ctypes.data
        L.check(L.lib().corro_process_multiple_changes(self.engine._h, self.bookie._h, descs, ncs, C.byref(s),
                                                       L.CORRO_MEM_HOST, C.byref(out)))
        res = Processed(known=[L.KNOWN.get(int(k), int(k)) for k in known[:ncs]])
        for i, cv1 in enumerate(changes):
            cs = cv1.changeset
            if isinstance(cs, Full):
                off = descs[i].change_off
                res.impactful.append([c for k, c in enumerate(cs.changes) if imp[off + k]])
            else:
                res.impactful.append([])
        res.ready = self.take_ready()
        return res

    def process_frames(self, buf, payload=0):
        """Wire bytes -> merge without leaving the GPU: decode length-delimited changeset frames
        on the device (corro_decode_frames, CORRO_MEM_DEVICE, with the kept frames' headers built on
        the device too) and hand the decoded batch and headers to process_multiple_changes where
        they lie (CORRO_MEM_DEVICE_HEADERS: no change or header crosses PCIe again; the known
        outcomes come back once). Frames with a non-zero decode status are not applied. Returns
        (Processed over the applied frames, with .impact = per-change impactful flags as a CUDA
        uint8 tensor, per-frame decode status)."""
        import torch
        dec = self.engine.decode_frames(buf, payload, device=True, device_headers=True)
        nk = dec["n_dev"]
        self.site_ids = dict(enumerate(self.engine.site_ids()))   # the decoder may have registered sites
        ch = dec["changes"]
        n = int(ch["pk"].shape[0])
        s = L.Changes()
        s.n = n
        for k, a in ch.items():
            if k == "val_data":
                s.val_data, s.val_data_len = a.data_ptr(), int(a.numel())
            else:
                setattr(s, k, a.data_ptr() if n else None)
        known = torch.zeros(max(1, nk), dtype=torch.int32, device="cuda")
        imp = torch.zeros(max(1, n), dtype=torch.uint8, device="cuda")
        out = L.ProcessOut()
        out.known = known.data_ptr()
        out.impactful = imp.data_ptr()
        torch.cuda.current_stream().synchronize()
        L.check(L.lib().corro_process_multiple_changes(self.engine._h, self.bookie._h, C.c_void_p(dec["cs_dev"].data_ptr()),
                                                       nk, C.byref(s), L.CORRO_MEM_DEVICE_HEADERS, C.byref(out)))
        res = Processed(known=[L.KNOWN.get(int(k), int(k)) for k in known[:nk].cpu().tolist()])
        res.impact = imp[:n]
        res.ready = self.take_ready()
        return res, dec["status"]

    def take_ready(self):
        c = C.c_uint64()
        L.check(L.lib().corro_bookie_take_ready(self.bookie._h, None, None, 0, C.byref(c)))
        if c.value == 0:
            return []
        a = np.zeros((c.value, 16), np.uint8)
        v = np.zeros(c.value, np.uint64)
        L.check(L.lib().corro_bookie_take_ready(self.bookie._h, a.ctypes.data, v.ctypes.data, c.value, C.byref(c)))
        return [(bytes(a[k]), int(v[k])) for k in range(c.value)]

    def process_fully_buffered_changes(self, actor, version):
        r = C.c_int()
        L.check(L.lib().corro_process_fully_buffered(self.engine._h, self.bookie._h, actor, version, C.byref(r)))
        return bool(r.value)

    def generate_sync(self):
        lib = L.lib()
        st = L.SyncState()
        L.check(lib.corro_generate_sync(self.bookie._h, self.actor_id, C.byref(st), 0))
        na, nn, npr, ns = st.n_actors, st.n_need, st.n_partials, st.n_pseqs
        bufs = {"actor_ids": np.zeros(max(1, 16 * na), np.uint8), "heads": np.zeros(max(1, na), np.uint64),
                "need_off": np.zeros(na + 1, np.uint64), "need_start": np.zeros(max(1, nn), np.uint64),
                "need_end": np.zeros(max(1, nn), np.uint64), "partial_off": np.zeros(na + 1, np.uint64),
                "partial_ver": np.zeros(max(1, npr), np.uint64), "pseq_off": np.zeros(npr + 1, np.uint64),
                "pseq_start": np.zeros(max(1, ns), np.uint64), "pseq_end": np.zeros(max(1, ns), np.uint64)}
        for k, a in bufs.items():
            setattr(st, k, a.ctypes.data)
        L.check(lib.corro_generate_sync(self.bookie._h, self.actor_id, C.byref(st), 1))
        state = SyncStateV1(actor_id=self.actor_id)
        for i in range(na):
            a = bytes(bufs["actor_ids"][16 * i:16 * i + 16])
            state.heads[a] = int(bufs["heads"][i])
            need = [(int(bufs["need_start"][k]), int(bufs["need_end"][k]))
                    for k in range(int(bufs["need_off"][i]), int(bufs["need_off"][i + 1]))]
            if need:
                state.need[a] = need
            for p in range(int(bufs["partial_off"][i]), int(bufs["partial_off"][i + 1])):
                seqs = [(int(bufs["pseq_start"][k]), int(bufs["pseq_end"][k]))
                        for k in range(int(bufs["pseq_off"][p]), int(bufs["pseq_off"][p + 1]))]
                state.partial_need.setdefault(a, {})[int(bufs["partial_ver"][p])] = seqs
        return state
