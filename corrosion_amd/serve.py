"""Server side of sync: answering a peer's SyncNeedV1 with changesets from the device state.

Mirrors corro-agent/src/api/peer/mod.rs `handle_need` (:371-727) and `send_change_chunks`
(:729-789), and corro-types/src/change.rs `Change::estimated_byte_size` (:34-49) and
`ChunkedChanges` (:66-178). The row lookups — the GROUP BY db_version query (:385-394) and the
per-version / per-seq-range row queries (:423-431, :603-611) — run on the GPU through
corro_extract_changes (csrc/extract.hip), batched over every need of the call. Buffered (partial)
versions and the gap bookkeeping come from the host Bookie (csrc/agent.cpp), as they come from
__corro_buffered_changes / __corro_seq_bookkeeping / __corro_bookkeeping_gaps in the reference.
"""
import ctypes as C
import struct

import numpy as np

from . import _lib as L
from .agent import Change, ChangeV1, Empty, Full
from .sync import Full as NeedFull, Partial as NeedPartial

MAX_CHANGES_BYTES_PER_MESSAGE = 8 * 1024   # peer/mod.rs:365
SEQ_ALL = (0, 0xFFFFFFFF)


# ---- change.rs / pubsub.rs size arithmetic --------------------------------------------------

def num_bytes_needed_i32(val):
    """pubsub.rs num_bytes_needed_i32 — including its `val * 0xFF != 0` test for the last byte,
    which is non-zero for every non-zero val (255 is odd, so the wrapping product is 0 only at 0)."""
    v = val & 0xFFFFFFFF
    if v & 0xFF000000:
        return 4
    if v & 0x00FF0000:
        return 3
    if v & 0x0000FF00:
        return 2
    return 1 if v != 0 else 0


def num_bytes_needed_i64(val):
    v = val & 0xFFFFFFFFFFFFFFFF
    if v & 0xFF00000000000000:
        return 8
    if v & 0x00FF000000000000:
        return 7
    if v & 0x0000FF0000000000:
        return 6
    if v & 0x000000FF00000000:
        return 5
    return num_bytes_needed_i32(v & 0xFFFFFFFF)


def packed_pk_len(pk):
    """len(pack_columns([Integer(pk)])) (pubsub.rs:2304-2358): count byte + type byte + int bytes."""
    return 2 + num_bytes_needed_i64(pk)


def value_size(val):
    """SqliteValue::estimated_byte_size (corro-api-types/src/lib.rs:524-532)."""
    if val is None:
        return 1 + 1
    if isinstance(val, (bool, int, float)):
        return 1 + 8
    b = val.encode() if isinstance(val, str) else bytes(val)
    return 1 + 4 + len(b)


def estimated_byte_size(ch):
    """Change::estimated_byte_size (change.rs:34-49)."""
    pk_len = len(ch.pk) if isinstance(ch.pk, (bytes, bytearray)) else packed_pk_len(ch.pk)
    return len(ch.table) + pk_len + len(ch.cid) + value_size(ch.val) + 8 + 8 + 8 + 16 + 8 + 8


class ChunkedChanges:
    """change.rs:66-178: yields (changes, (start_seq, end_seq)) chunks of at most ~max_buf_size
    estimated bytes; the last chunk always ends at last_seq (even when empty)."""

    def __init__(self, it, start_seq, last_seq, max_buf_size, size=estimated_byte_size):
        self._it = iter(it)
        self._peek = []
        self.last_pushed_seq = 0
        self.last_start_seq = start_seq
        self.last_seq = last_seq
        self.max_buf_size = max_buf_size
        self.done = False
        self._size = size

    def _next_item(self):
        if self._peek:
            return self._peek.pop()
        return next(self._it, None)

    def _has_next(self):
        if not self._peek:
            x = next(self._it, None)
            if x is None:
                return False
            self._peek.append(x)
        return True

    def __iter__(self):
        return self

    def __next__(self):
        if self.done:
            raise StopIteration
        changes, buffered = [], 0
        while True:
            ch = self._next_item()
            if ch is None:
                break
            self.last_pushed_seq = ch.seq
            buffered += self._size(ch)
            changes.append(ch)
            if self.last_pushed_seq == self.last_seq:
                break
            if buffered >= self.max_buf_size:
                start = self.last_start_seq
                if not self._has_next():
                    break
                self.last_start_seq = self.last_pushed_seq + 1
                return changes, (start, self.last_pushed_seq)
        self.done = True
        return changes, (self.last_start_seq, self.last_seq)


def send_change_chunks(out, chunked, actor_id, version, last_seq, ts):
    """peer/mod.rs:729-789 without the channel: append Changeset::Full messages to `out`
    (an empty first-and-only chunk covering 0..=last_seq is dropped, :746-748)."""
    for changes, seqs in chunked:
        if not changes and seqs[0] == 0 and seqs[1] == last_seq:
            return
        out.append(ChangeV1(actor_id, Full(version=version, changes=changes, seqs=seqs, last_seq=last_seq, ts=ts)))


# ---- rows -> Change objects -------------------------------------------------------------------

def _decode_value(vt, v0, v1, ln, long_bytes=None):
    vt = int(vt)
    if vt in (3, 4) and int(ln) == L.CORRO_VAL_LONG:  # a long value: its bytes from the arena / bookie
        b = long_bytes()
        return b.decode() if vt == 3 else b
    if vt == 1:
        return struct.unpack("<q", struct.pack("<Q", int(v0)))[0]
    if vt == 2:
        return struct.unpack("<d", struct.pack("<Q", int(v0)))[0]
    if vt in (3, 4):
        b = (int(v0).to_bytes(8, "big") + int(v1).to_bytes(8, "big"))[: int(ln)]
        return b.decode() if vt == 3 else b
    return None


def rows_to_changes(engine, site_ids, rows, lo, hi, long_bytes=None):
    """crsql_changes rows [lo, hi) -> Change objects (table / cid names from the engine schema).
    long_bytes(k): the bytes of row k's long value (default: its val1 handle in the engine's arena)."""
    out = []
    if long_bytes is None:
        def long_bytes(k):
            return engine.value_bytes([int(rows["val1"][k])])[0]
    for k in range(lo, hi):
        tc = int(rows["table_cid"][k])
        t, cid = tc >> 16, tc & 0xFFFF
        name, cols = engine.schema[t]
        pk = int(rows["pk"][k])
        if name in engine.interned:  # the canonical packed pk of the row (cr-sqlite's t__crsql_pks)
            pk = engine.pk_bytes(t, [pk])[0]
        out.append(Change(table=name, pk=pk, cid="-1" if cid == 0 else cols[cid - 1],
                          val=_decode_value(rows["val_type"][k], rows["val0"][k], rows["val1"][k], rows["val_len"][k],
                                            lambda: long_bytes(k)),
                          col_version=int(rows["col_version"][k]), db_version=int(rows["db_version"][k]),
                          seq=int(rows["seq"][k]), site_id=site_ids[int(rows["site"][k])], cl=int(rows["cl"][k])))
    return out


# ---- bookie probes ------------------------------------------------------------------------------

def _buffered_versions(bookie, actor, s, e):
    c = C.c_uint64()
    L.check(L.lib().corro_bookie_buffered_versions(bookie._h, actor, s, e, None, 0, C.byref(c)))
    if not c.value:
        return []
    v = np.zeros(c.value, np.uint64)
    L.check(L.lib().corro_bookie_buffered_versions(bookie._h, actor, s, e, v.ctypes.data, c.value, C.byref(c)))
    return [int(x) for x in v]


def _seq_bookkeeping(bookie, actor, version):
    c, last, ts = C.c_uint64(), C.c_int64(), C.c_uint64()
    L.check(L.lib().corro_bookie_seq_bookkeeping(bookie._h, actor, version, None, None, 0, C.byref(c),
                                                 C.byref(last), C.byref(ts)))
    if last.value < 0 or not c.value:
        return []
    s = np.zeros(c.value, np.uint64)
    e = np.zeros(c.value, np.uint64)
    L.check(L.lib().corro_bookie_seq_bookkeeping(bookie._h, actor, version, s.ctypes.data, e.ctypes.data, c.value,
                                                 C.byref(c), C.byref(last), C.byref(ts)))
    return [((int(s[i]), int(e[i])), int(last.value), int(ts.value)) for i in range(c.value)]


def _buffered_rows(bookie, actor, version, s, e):
    c = C.c_uint64()
    L.check(L.lib().corro_bookie_buffered(bookie._h, actor, version, s, e, None, 0, C.byref(c)))
    from .engine import ROW_FIELDS
    rows = {k: np.zeros(max(1, c.value), dt) for k, dt in ROW_FIELDS.items()}
    r = L.Rows()
    for k, a in rows.items():
        setattr(r, k, a.ctypes.data)
    L.check(L.lib().corro_bookie_buffered(bookie._h, actor, version, s, e, C.byref(r), c.value, C.byref(c)))
    return rows, c.value


def _buffered_long(bookie, actor, version, rows):
    """long_bytes for rows_to_changes over buffered rows: the bookie keeps their bytes."""
    def get(k):
        n = C.c_uint64()
        seq = int(rows["seq"][k])
        L.check(L.lib().corro_bookie_buffered_value(bookie._h, actor, version, seq, None, 0, C.byref(n)))
        buf = C.create_string_buffer(max(1, n.value))
        L.check(L.lib().corro_bookie_buffered_value(bookie._h, actor, version, seq, buf, n.value, C.byref(n)))
        return buf.raw[:n.value]
    return get


def _in_ranges(ranges, v):
    return any(s <= v <= e for s, e in ranges)


def _subtract(ranges, holes):
    """[(s, e)] - [(s, e)] over integers, ascending, coalesced (RangeInclusiveSet::remove)."""
    out = []
    for s, e in ranges:
        cur = [(s, e)]
        for hs, he in holes:
            nxt = []
            for a, b in cur:
                if he < a or hs > b:
                    nxt.append((a, b))
                    continue
                if a < hs:
                    nxt.append((a, hs - 1))
                if he < b:
                    nxt.append((he + 1, b))
            cur = nxt
        out.extend(cur)
    out.sort()
    merged = []
    for a, b in out:
        if merged and a <= merged[-1][1] + 1:
            merged[-1] = (merged[-1][0], max(merged[-1][1], b))
        else:
            merged.append((a, b))
    return merged


# ---- handle_need ----------------------------------------------------------------------------

def handle_needs(agent, needs, max_buf_size=MAX_CHANGES_BYTES_PER_MESSAGE):
    """handle_need (peer/mod.rs:371-727) for a list of (actor_id, SyncNeedV1) at once.

    Change.site_id comes from the engine's site table (ordinal -> 16 bytes). Returns, per need,
    the list of ChangeV1 messages in the order the reference sends them. The crsql_changes
    queries of every need run as ONE batched device extraction."""
    eng = agent.engine
    site_ids = dict(enumerate(eng.site_ids()))
    # one extraction entry per crsql_changes query
    ent_site, ent_s, ent_e, ent_ss, ent_se, owner = [], [], [], [], [], []
    plan = []
    for i, (actor, need) in enumerate(needs):
        site = agent.site(actor)
        if isinstance(need, NeedFull):
            plan.append(("full", len(ent_site)))
            ent_site.append(site); ent_s.append(need.start); ent_e.append(need.end)
            ent_ss.append(SEQ_ALL[0]); ent_se.append(SEQ_ALL[1]); owner.append(i)
        elif isinstance(need, NeedPartial):
            first = len(ent_site)
            for s, e in [SEQ_ALL] + [tuple(r) for r in need.seqs]:
                ent_site.append(site); ent_s.append(need.version); ent_e.append(need.version)
                ent_ss.append(max(0, min(s, 0xFFFFFFFF))); ent_se.append(max(0, min(e, 0xFFFFFFFF))); owner.append(i)
            plan.append(("partial", first))
        else:
            plan.append(("none", -1))
    res = None
    if ent_site:
        res = eng.extract_changes({"site": np.array(ent_site, np.uint32), "start": np.array(ent_s, np.uint64),
                                   "end": np.array(ent_e, np.uint64), "seq_start": np.array(ent_ss, np.uint32),
                                   "seq_end": np.array(ent_se, np.uint32)})

    def groups(k):
        g0, g1 = int(res["grp_off"][k]), int(res["grp_off"][k + 1])
        return [(int(res["version"][g]), int(res["last_seq"][g]), int(res["ts"][g]), int(res["grp_row_off"][g]),
                 int(res["grp_rows"][g])) for g in range(g0, g1)]

    out_all = []
    for (actor, need), (kind, k) in zip(needs, plan):
        out, empties = [], []
        if kind == "full":
            found = set()
            for version, last_seq, ts, ro, rn in groups(k):    # db_version DESC (:385-394)
                found.add(version)
                chunks = ChunkedChanges(rows_to_changes(eng, site_ids, res["rows"], ro, ro + rn), 0, last_seq,
                                        max_buf_size)
                send_change_chunks(out, chunks, actor, version, last_seq, ts)
            unprocessed = _subtract([(need.start, need.end)], [(v, v) for v in sorted(found)])
            gaps = agent.bookie.needed(actor)
            for s, e in unprocessed:                           # :458-542
                buffered = _buffered_versions(agent.bookie, actor, s, e)
                for v in buffered:
                    for (rs, re_), last_seq, ts in _seq_bookkeeping(agent.bookie, actor, v):
                        rows, m = _buffered_rows(agent.bookie, actor, v, rs, re_)
                        chg = rows_to_changes(eng, site_ids, rows, 0, m, _buffered_long(agent.bookie, actor, v, rows))
                        send_change_chunks(out, ChunkedChanges(chg, rs, re_, max_buf_size), actor, v, last_seq, ts)
                empties += _subtract([(s, e)], gaps + [(v, v) for v in buffered])
        elif kind == "partial":
            g = groups(k)
            if g:                                              # :554-597
                version, last_seq, ts, _, _ = g[0]
                for j, (s, e) in enumerate(need.seqs):
                    _, _, _, ro, rn = groups(k + 1 + j)[0]
                    chunks = ChunkedChanges(rows_to_changes(eng, site_ids, res["rows"], ro, ro + rn), s, e, max_buf_size)
                    send_change_chunks(out, chunks, actor, version, last_seq, ts)
            else:                                              # :598-712
                v = need.version
                in_gaps = _in_ranges(agent.bookie.needed(actor), v)
                buffered = bool(_buffered_versions(agent.bookie, actor, v, v))
                if not buffered and not in_gaps:
                    empties.append((v, v))
                if buffered:
                    for qs, qe in need.seqs:
                        for (rs, re_), last_seq, ts in _seq_bookkeeping(agent.bookie, actor, v):
                            hit = (qs <= rs <= qe) or (rs <= qs and re_ >= qe) or (rs <= qe and re_ >= qe) or \
                                  (qs <= re_ <= qe)
                            if not hit:
                                continue
                            s, e = max(rs, qs), min(re_, qe)
                            rows, m = _buffered_rows(agent.bookie, actor, v, s, e)
                            chg = rows_to_changes(eng, site_ids, rows, 0, m,
                                                  _buffered_long(agent.bookie, actor, v, rows))
                            send_change_chunks(out, ChunkedChanges(chg, s, e, max_buf_size), actor, v, last_seq, ts)
        for s, e in _subtract(empties, []):                    # :715-724
            out.append(ChangeV1(actor, Empty(versions=(s, e), ts=None)))
        out_all.append(out)
    return out_all


def handle_need(agent, actor_id, need, max_buf_size=MAX_CHANGES_BYTES_PER_MESSAGE):
    return handle_needs(agent, [(actor_id, need)], max_buf_size)[0]
