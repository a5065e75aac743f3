"""Caller of the merge path: the batching loop of corro-agent's `handle_changes`
(crates/corro-agent/src/agent/handlers.rs:548-786), restated as a synchronous state machine.

The reference is one tokio task: changes arrive on a channel, are filtered (own actor :667-669,
seen-cache :671-686, already booked :711-727), queued with a processing cost, and handed to
`process_multiple_changes` in batches of at least `apply_queue_len` cost units (:578-611), with at
most MAX_CONCURRENT = 5 batches in flight (:561) and a timer that flushes a short queue every
`apply_queue_timeout` ms (:632-655). A full queue (`processing_queue_len`) drops its oldest entry
(:729-751). Here each of the loop's events is a method — `recv` (a change arrives), `tick` (the
timer fires), `job_done` (a batch finished) — and each returns the batches the loop spawns next,
in order; the caller applies them (one writer: `Agent.process_multiple_changes`) and reports
completion with `job_done`. The HLC clock update from the change's timestamp (:689-708), metrics
and rebroadcast (:763-775) are transport concerns outside the merge path and are not modelled.

Reference quirks kept on purpose (tests/test_queue.py):
  * `Changeset::EmptySet` reports the dummy version range 0..=0 (broadcast.rs:171-179), so the
    seen-cache keys it under version 0;
  * dropping the oldest queued change clears its seen entries under the *arriving* change's
    actor id (handlers.rs:736 uses `change.actor_id`, not the dropped one's);
  * the seen cache is an IndexMap: removing an entry swaps the last entry into its slot
    (indexmap 2.1 `OccupiedEntry::remove_entry` = `swap_remove_entry`), and trimming keeps the
    newest `max(10, len/10)` entries by position (`split_off`, :651-654).
"""
from collections import deque

from .agent import Empty, EmptySet, Full

MAX_CONCURRENT = 5                 # handlers.rs:561
DEFAULT_APPLY_QUEUE_LEN = 50       # corro-types/src/config.rs:15-17 (perf.apply_queue_len)
DEFAULT_PROCESSING_QUEUE_LEN = 20000  # config.rs:23-25 (perf.processing_queue_len)
DEFAULT_APPLY_QUEUE_TIMEOUT_MS = 10   # config.rs:45-47 (perf.apply_queue_timeout)


def versions(cs):
    """Changeset::versions (broadcast.rs:171-179): inclusive (start, end)."""
    if isinstance(cs, Empty):
        return tuple(cs.versions)
    if isinstance(cs, EmptySet):
        return (0, 0)
    return (cs.version, cs.version)


def seqs(cs):
    """Changeset::seqs (broadcast.rs:199-205)."""
    return tuple(cs.seqs) if isinstance(cs, Full) else None


def processing_cost(cs):
    """Changeset::processing_cost (broadcast.rs:182-193)."""
    if isinstance(cs, Empty):
        return min(cs.versions[1] - cs.versions[0] + 1, 20)
    if isinstance(cs, EmptySet):
        return sum(min(e - s + 1, 20) for s, e in cs.versions)
    return len(cs.changes)


class SeqSet:
    """rangemap RangeInclusiveSet<CrsqlSeq>: disjoint ranges, touching ones coalesced (StepLite)."""

    def __init__(self):
        self.r = []  # sorted [start, end]

    def extend(self, rng):
        s, e = rng
        if e < s:
            return  # (rangemap panics on an empty range; nothing to add)
        out = []
        for a, b in self.r:
            if b + 1 < s or e + 1 < a:
                out.append([a, b])
            else:
                s, e = min(s, a), max(e, b)
        out.append([s, e])
        self.r = sorted(out)

    def remove(self, rng):
        s, e = rng
        out = []
        for a, b in self.r:
            if b < s or e < a:
                out.append([a, b])
                continue
            if a < s:
                out.append([a, s - 1])
            if e < b:
                out.append([e + 1, b])
        self.r = out

    def contains_all(self, rng):
        """`seqs.all(|seq| set.contains(&seq))` for the inclusive range (vacuous when empty)."""
        s, e = rng
        if e < s:
            return True
        return any(a <= s and e <= b for a, b in self.r)

    def ranges(self):
        return [tuple(x) for x in self.r]


class SeenCache:
    """IndexMap<(ActorId, CrsqlDbVersion), RangeInclusiveSet<CrsqlSeq>> with indexmap 2.1 order."""

    def __init__(self):
        self.keys = []
        self.vals = []
        self.index = {}

    def __len__(self):
        return len(self.keys)

    def __contains__(self, k):
        return k in self.index

    def get(self, k):
        i = self.index.get(k)
        return None if i is None else self.vals[i]

    def entry_or_default(self, k):
        i = self.index.get(k)
        if i is None:
            i = len(self.keys)
            self.keys.append(k)
            self.vals.append(SeqSet())
            self.index[k] = i
        return self.vals[i]

    def swap_remove(self, k):
        i = self.index.pop(k)
        last = len(self.keys) - 1
        if i != last:
            self.keys[i], self.vals[i] = self.keys[last], self.vals[last]
            self.index[self.keys[i]] = i
        self.keys.pop()
        self.vals.pop()

    def keep_last(self, n):
        """`*self = self.split_off(len - n)`."""
        cut = len(self.keys) - n
        self.keys, self.vals = self.keys[cut:], self.vals[cut:]
        self.index = {k: i for i, k in enumerate(self.keys)}


class ChangeQueue:
    """handle_changes' loop state: queue, cost, in-flight batches and the seen cache.

    actor_id: this node's actor (its own changes are ignored); contains_all(actor, versions, seqs)
    answers the Bookie check (`Booked::contains_all`, agent.rs:1380-1390), e.g. `Bookie.contains_all`.
    """

    def __init__(self, actor_id, contains_all, apply_queue_len=DEFAULT_APPLY_QUEUE_LEN,
                 processing_queue_len=DEFAULT_PROCESSING_QUEUE_LEN, max_concurrent=MAX_CONCURRENT, clock=None):
        self.actor_id = bytes(actor_id)
        self.contains_all = contains_all
        self.max_changes_chunk = apply_queue_len
        self.max_queue_len = processing_queue_len
        self.max_concurrent = max_concurrent
        self.max_seen_cache_len = processing_queue_len
        self.keep_seen_cache_size = max(10, processing_queue_len // 10) if processing_queue_len > 10 else 0
        self.clock = clock or (lambda: 0)
        self.queue = deque()     # (ChangeV1, source, queued_at)
        self.buf_cost = 0
        self.in_flight = 0
        self.seen = SeenCache()
        self.dropped = 0

    # -- loop top (handlers.rs:578-611) ------------------------------------------------------------
    def _spawn_ready(self):
        out = []
        while ((self.buf_cost >= self.max_changes_chunk or (self.queue and self.in_flight == 0))
               and self.in_flight < self.max_concurrent):
            buf, tmp_cost = [], 0
            while self.queue:
                item = self.queue.popleft()
                tmp_cost += processing_cost(item[0].changeset)
                buf.append(item)
                if tmp_cost >= self.max_changes_chunk:
                    break
            if not buf:
                break
            self.in_flight += 1
            out.append(buf)
            self.buf_cost -= tmp_cost
        return out

    # -- select! arms -------------------------------------------------------------------------------
    def job_done(self):
        """A spawned process_multiple_changes finished (join_next arm, :616-622)."""
        if self.in_flight <= 0:
            raise ValueError("no batch in flight")
        self.in_flight -= 1
        return self._spawn_ready()

    def tick(self):
        """apply_queue_timeout elapsed (max_wait arm, :632-657)."""
        out = []
        if self.buf_cost < self.max_changes_chunk and self.queue and self.in_flight < self.max_concurrent:
            out.append(list(self.queue))
            self.queue.clear()
            self.in_flight += 1
            self.buf_cost = 0
        if len(self.seen) > self.max_seen_cache_len:
            self.seen.keep_last(self.keep_seen_cache_size)
        return out + self._spawn_ready()

    def recv(self, change, source="sync"):
        """A (ChangeV1, ChangeSource) arrived on rx_changes (:664-783)."""
        cs = change.changeset
        actor = bytes(change.actor_id)
        if actor == self.actor_id:
            return self._spawn_ready()
        sq = seqs(cs)
        vs = versions(cs)
        if sq is not None:
            got = self.seen.get((actor, vs[0]))
            if got is not None and got.contains_all(sq):
                return self._spawn_ready()
        elif all((actor, v) in self.seen for v in range(vs[0], vs[1] + 1)):
            return self._spawn_ready()
        if self.contains_all(actor, vs, sq):
            return self._spawn_ready()
        if len(self.queue) >= self.max_queue_len:
            dropped, _, _ = self.queue.popleft()
            dvs, dsq = versions(dropped.changeset), seqs(dropped.changeset)
            for v in range(dvs[0], dvs[1] + 1):
                k = (actor, v)  # sic: the arriving change's actor (handlers.rs:736)
                if k in self.seen:
                    if dsq is not None:
                        self.seen.get(k).remove(dsq)
                    else:
                        self.seen.swap_remove(k)
            self.buf_cost -= processing_cost(dropped.changeset)
            self.dropped += 1
        for v in range(vs[0], vs[1] + 1):
            e = self.seen.entry_or_default((actor, v))
            if sq is not None:
                e.extend(sq)
        self.queue.append((change, source, self.clock()))
        self.buf_cost += processing_cost(cs)
        return self._spawn_ready()
