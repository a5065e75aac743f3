"""CPU restatement of process_multiple_changes for the parity tests (TEST INFRASTRUCTURE: only
tests/ import it; the product path is csrc/agent.cpp + agent_dev.hip).

Follows /root/reference/crates/corro-agent/src/agent/util.rs:
  :704-739   pass 1: batch-local dedup of (actor, versions, seqs), then versions the actor's
             BookedVersions already contains_all (corro-types/src/agent.rs:1368-1390)
  :765-884   pass 2 per actor in ActorId byte order: versions already seen in this call (the
             RangeInclusiveMap of PartialVersion), empty versions (crsql_set_db_version only when
             end > the actor's max, :810-824), invalid seqs (:826-831), the SAVEPOINT per version
             (an unknown table/column rolls the version back, :839-860), incomplete versions buffered
             with their seq ranges merged (:1053-1186), complete versions merged
  :1218-1261 impactful: crsql_rows_impacted() is cumulative over the transaction while
             last_rows_impacted restarts at 0 per version
  :894-932   gap bookkeeping of every processed version range (insert_db, agent.rs:1108-1235)
over the oracle's own restatements: the merge fold (crsql_fold.c, pinned by the cr-sqlite KATs) and
the RangeInclusiveSet gap bookkeeping (ranges.c, pinned by agent.rs:1605-1868). Scope: Full, Empty
and EmptySet changesets, calls that commit (no UNIQUE-constraint rollback), changes given as
engine-encoded fields. EmptySet reports the dummy range 0..=0 (broadcast.rs:176), is complete and
empty (:218, :236) and has no seqs (:201); BookedVersions::contains_version(0) holds for every actor
(max.unwrap_or_default() >= 0 and no gap holds 0, agent.rs:1353-1361), so pass 1's contains_all
(util.rs:724-733) always skips it: an EmptySet is never processed (known "skipped", no
crsql_set_db_version, no gap bookkeeping). The restatement keeps the reference's full control flow
for it anyway, so a bookkeeping state with 0 in a gap would process it as the reference does.
"""
from . import oracle as O

UNKNOWN = 0xFFFFFFFF


def _rs_insert(rs, s, e):
    """RangeInclusiveSet insert with coalescing of touching ranges (StepLite)."""
    out, placed = [], False
    for a, b in rs:
        if b + 1 < s:
            out.append((a, b))
        elif e + 1 < a:
            if not placed:
                out.append((s, e))
                placed = True
            out.append((a, b))
        else:
            s, e = min(s, a), max(e, b)
    if not placed:
        out.append((s, e))
    return sorted(out)


def _rs_contains_range(rs, s, e):
    return s <= e and any(a <= s and e <= b for a, b in rs)


def _rs_gaps(rs, s, e):
    out, x = [], s
    for a, b in sorted(rs):
        if b < x or a > e:
            continue
        if a > x:
            out.append((x, a - 1))
        x = max(x, b + 1)
        if x > e:
            return out
    if x <= e:
        out.append((x, e))
    return out


class Partial:
    def __init__(self, seqs, last_seq, ts):
        self.seqs, self.last_seq, self.ts = list(seqs), last_seq, ts


class ActorBook:
    def __init__(self):
        self.gaps = O.Booked()
        self.partials = {}   # version -> Partial

    def max(self):
        return self.gaps.max()

    def contains_all(self, s, e, seqs):
        if s > e:
            return True
        mx = self.max() or 0  # max.unwrap_or_default() (agent.rs:1353-1361)
        if e > mx:
            return False
        if any(not (b < s or a > e) for a, b in self.gaps.needed()):
            return False
        if seqs is None or seqs[0] > seqs[1]:
            return True
        return all(_rs_contains_range(p.seqs, *seqs) for v, p in self.partials.items() if s <= v <= e)


class Changeset:
    """One ChangeV1: kind 'full' (version, seqs, last_seq, ts, rows), 'empty' (versions) or 'empty_set'
    (versions: the list of ranges it carries; only its dummy 0..=0 takes part in the apply)."""

    def __init__(self, actor, kind, version=None, versions=None, seqs=None, last_seq=None, ts=0, rows=()):
        self.actor, self.kind, self.ts = bytes(actor), kind, ts
        self.version, self.versions, self.seqs, self.last_seq = version, versions, seqs, last_seq
        self.rows = list(rows)  # dicts of engine fields: pk, table_cid, col_version, db_version, cl, seq, site, val0

    def vrange(self):
        if self.kind == "empty_set":
            return (0, 0)  # Changeset::versions() dummy (broadcast.rs:176)
        return (self.version, self.version) if self.kind == "full" else tuple(self.versions)

    def complete(self):
        return self.kind != "full" or (self.seqs[0] == 0 and self.seqs[1] == self.last_seq)

    def empty(self):
        return self.kind != "full" or not self.rows


class AgentOracle:
    def __init__(self, site_ids):
        self.fold = O.Fold(site_ids)
        self.site_of = {bytes(s): i for i, s in enumerate(site_ids)}
        self.books = {}        # actor -> ActorBook
        self.seqbook = {}      # (actor, version) -> list of seq ranges
        self.buffered = {}     # (actor, version) -> {seq: row}
        self.set_dbv = {}      # site -> max version set by crsql_set_db_version
        self.ready = []

    def book(self, a):
        return self.books.setdefault(a, ActorBook())

    def process(self, changesets):
        """Returns (known per changeset, impactful flags per changeset's rows)."""
        n = len(changesets)
        known = ["skipped"] * n
        impactful = [[0] * len(c.rows) for c in changesets]
        seen, unknown = set(), {}
        for i, c in enumerate(changesets):                   # pass 1
            v = c.vrange()
            seqs = tuple(c.seqs) if c.kind == "full" else None
            key = (c.actor, v, seqs)
            if key in seen:
                continue
            seen.add(key)
            if self.book(c.actor).contains_all(v[0], v[1], seqs):
                continue
            unknown.setdefault(c.actor, []).append(i)
        applied, processed = [], {}
        for actor in sorted(unknown):                         # pass 2, ActorId order
            bk = self.book(actor)
            had = bk.max()
            local = []                                        # [(range, Partial or None)], later wins
            for i in unknown[actor]:
                c = changesets[i]
                v = c.vrange()
                seqs = tuple(c.seqs) if c.kind == "full" else None

                def seen_v(x):
                    for (a, b), p in reversed(local):
                        if a <= x <= b:
                            return True, p
                    return False, None
                ok = True
                for x in range(v[0], v[1] + 1):
                    hit, p = seen_v(x)
                    if not hit or (seqs is not None and p is not None and not _rs_contains_range(p.seqs, *seqs)):
                        ok = False
                        break
                if ok:
                    continue
                partial = None
                if c.complete() and c.empty():
                    if had is None or v[1] > had:
                        self.set_dbv[c.actor] = max(self.set_dbv.get(c.actor, 0), v[1])
                    known[i] = "cleared"
                else:
                    if seqs is not None and seqs[1] < seqs[0]:
                        continue
                    if any(r["table_cid"] == UNKNOWN for r in c.rows):
                        known[i] = -5
                        continue
                    if c.complete():
                        applied.append(i)
                        known[i] = "current"
                    else:
                        partial = self._incomplete(c)
                        if partial is None:
                            known[i] = -1
                            continue
                        known[i] = "partial"
                local.append((v, partial))
                processed.setdefault(actor, []).append((v, partial))
        # the merge, with the cumulative crsql_rows_impacted() rule
        rows = [r for i in applied for r in changesets[i].rows]
        imp = self.fold.apply(_batch(rows, [changesets[i].ts for i in applied for _ in changesets[i].rows])) \
            if rows else []
        cum, k = 0, 0
        for i in applied:
            last, anyhit = 0, False
            for j in range(len(changesets[i].rows)):
                cum += int(imp[k])
                k += 1
                hit = cum > last
                last = cum
                if hit:
                    impactful[i][j] = 1
                    anyhit = True
            known[i] = "current" if anyhit else "cleared"
            self.buffered.pop((changesets[i].actor, changesets[i].version), None)
            self.seqbook.pop((changesets[i].actor, changesets[i].version), None)
        # gap bookkeeping, then partials
        for actor, lst in processed.items():
            bk = self.book(actor)
            vs = []
            for v, _p in lst:
                vs = _rs_insert(vs, v[0], v[1])
            assert bk.gaps.insert_db(vs) == 0
            for v, p in lst:
                if p is None:
                    continue
                cur = bk.partials.get(v[0])
                if cur is None:
                    bk.partials[v[0]] = p
                    cur = p
                else:
                    for a, b in p.seqs:
                        cur.seqs = _rs_insert(cur.seqs, a, b)
                if not _rs_gaps(cur.seqs, 0, cur.last_seq):
                    self.ready.append((actor, v[0]))
        return known, impactful

    def _incomplete(self, c):
        """process_incomplete_version (util.rs:1053-1186): buffer the rows, merge the seq range."""
        key = (c.actor, c.version)
        ranges = list(self.seqbook.get(key, []))
        s, e = c.seqs
        merged, keep = [], []
        for a, b in ranges:
            hit = (s <= a <= e) or (a <= s and b >= e) or (a <= e <= b) or (s <= b <= e) or \
                  (a == e + 1 and b != 0) or (s > 0 and b == s - 1)
            (merged if hit else keep).append((a, b))
        m = []
        for a, b in merged + [(s, e)]:
            m = _rs_insert(m, a, b)
        if len(m) != 1:
            return None
        self.seqbook[key] = keep + m
        buf = self.buffered.setdefault(key, {})
        for r in c.rows:
            buf.setdefault(r["seq"], r)
        return Partial(m, c.last_seq, c.ts)

    def export(self):
        return self.fold.export()

    def needed(self, actor):
        return self.book(actor).gaps.needed() if actor in self.books else []

    def last(self, actor):
        return self.book(actor).max() if actor in self.books else None


def _batch(rows, ts):
    import numpy as np
    keys = {"pk": np.uint64, "table_cid": np.uint32, "col_version": np.int64, "db_version": np.int64,
            "cl": np.uint32, "seq": np.uint32, "site": np.uint32, "val0": np.uint64, "val_type": np.uint8}
    b = {k: np.array([r.get(k, 1) for r in rows], dt) for k, dt in keys.items()}
    b["ts"] = np.array(ts, np.uint64)
    return b
