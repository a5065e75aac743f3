"""handle_changes' batching loop (corrosion_amd/queue.py) on CPU, against the reference's
test_loadshed_handle_changes (handlers.rs:931-1000) and the loop's documented rules and quirks
(handlers.rs:548-786, broadcast.rs:171-205)."""
from corrosion_amd.agent import Change, ChangeV1, Empty, EmptySet, Full
from corrosion_amd.queue import ChangeQueue, SeqSet, processing_cost, versions

ME = b"\x01" * 16
OTHER = b"\x02" * 16


def full(actor, version, n=1, seqs=None, last_seq=None):
    chs = [Change("tests", version, "text", "x", 1, version, i, actor, 1) for i in range(n)]
    seqs = seqs or (0, n - 1)
    return ChangeV1(actor, Full(version, chs, seqs, last_seq if last_seq is not None else n - 1))


class Booked:
    """Stand-in for the Bookie: versions applied by finished batches."""

    def __init__(self):
        self.done = set()

    def contains_all(self, actor, vs, sq):
        return all((actor, v) in self.done for v in range(vs[0], vs[1] + 1))

    def apply(self, batch):
        for cv1, _, _ in batch:
            s, e = versions(cv1.changeset)
            for v in range(s, e + 1):
                self.done.add((bytes(cv1.actor_id), v))


def test_loadshed_kat():
    # apply_queue_len 1, processing_queue_len 3; the write connection is held, so the five
    # batches for versions 10..6 stay in flight; 5, 4, 3 queue; 2 and 1 displace 5 and 4.
    bk = Booked()
    q = ChangeQueue(ME, bk.contains_all, apply_queue_len=1, processing_queue_len=3)
    running = []
    for i in range(10, 0, -1):
        running += q.recv(full(OTHER, i))
    assert [b[0][0].changeset.version for b in running] == [10, 9, 8, 7, 6]
    assert [c.changeset.version for c, _, _ in q.queue] == [3, 2, 1]
    assert q.dropped == 2
    while running:  # the connection is released: batches finish one by one
        b = running.pop(0)
        bk.apply(b)
        running += q.job_done()
    ok = lambda s, e: bk.contains_all(OTHER, (s, e), None)
    assert ok(6, 10) and ok(1, 3)
    assert not ok(5, 5) and not ok(4, 4)


def test_costs():
    assert processing_cost(full(OTHER, 1, n=7).changeset) == 7
    assert processing_cost(Empty((3, 10))) == 8
    assert processing_cost(Empty((1, 100))) == 20
    assert processing_cost(EmptySet([(1, 5), (10, 100)], 0)) == 25
    assert versions(EmptySet([(4, 9)], 0)) == (0, 0)  # dummy range (broadcast.rs:174-176)


def test_batches_reach_chunk_cost():
    q = ChangeQueue(ME, lambda *a: False, apply_queue_len=10)
    out = q.recv(full(OTHER, 1, n=4))  # nothing in flight: a non-empty queue spawns at once
    assert len(out) == 1 and q.in_flight == 1
    assert q.recv(full(OTHER, 2, n=4)) == [] and q.recv(full(OTHER, 3, n=4)) == []
    out = q.recv(full(OTHER, 4, n=4))  # cost 12 >= 10: one batch of 3 changesets (4+4+4)
    assert [[c.changeset.version for c, _, _ in b] for b in out] == [[2, 3, 4]]
    assert q.buf_cost == 0 and q.in_flight == 2


def test_tick_flushes_short_queue():
    q = ChangeQueue(ME, lambda *a: False, apply_queue_len=50)
    assert len(q.recv(full(OTHER, 1))) == 1
    assert q.recv(full(OTHER, 2)) == [] and q.recv(full(OTHER, 3)) == []
    out = q.tick()
    assert [[c.changeset.version for c, _, _ in b] for b in out] == [[2, 3]]
    assert q.buf_cost == 0 and not q.queue


def test_max_concurrent():
    q = ChangeQueue(ME, lambda *a: False, apply_queue_len=1)
    got = []
    for v in range(1, 9):
        got += q.recv(full(OTHER, v))
    assert len(got) == 5 and q.in_flight == 5 and len(q.queue) == 3
    assert q.tick() == []  # no capacity
    assert len(q.job_done()) == 1


def test_filters():
    booked = {(OTHER, 7)}
    q = ChangeQueue(ME, lambda a, vs, sq: all((a, v) in booked for v in range(vs[0], vs[1] + 1)),
                    apply_queue_len=100)
    q.in_flight = 1  # keep everything queued
    q.recv(full(ME, 1))                      # own actor
    q.recv(full(OTHER, 7))                   # already booked
    q.recv(full(OTHER, 2, n=3))              # queued
    q.recv(full(OTHER, 2, n=2, seqs=(0, 1), last_seq=2))  # seqs 0..=1 already seen for v2
    q.recv(full(OTHER, 3, n=1, seqs=(0, 0), last_seq=4))
    q.recv(full(OTHER, 3, n=2, seqs=(0, 1), last_seq=4))  # seq 1 not seen yet: queued
    q.recv(ChangeV1(OTHER, Empty((10, 12))))
    q.recv(ChangeV1(OTHER, Empty((11, 12))))  # every version seen
    q.recv(ChangeV1(OTHER, Empty((12, 13))))  # 13 not seen: queued
    assert [(versions(c.changeset), len(getattr(c.changeset, "changes", []))) for c, _, _ in q.queue] == [
        ((2, 2), 3), ((3, 3), 1), ((3, 3), 2), ((10, 12), 0), ((12, 13), 0)]
    assert q.seen.get((OTHER, 3)).ranges() == [(0, 1)]
    # EmptySet is keyed under its dummy version 0, so a second EmptySet is filtered
    q.recv(ChangeV1(OTHER, EmptySet([(20, 30)], 0)))
    q.recv(ChangeV1(OTHER, EmptySet([(40, 50)], 0)))
    assert len(q.queue) == 6


def test_drop_uses_arriving_actor():
    a2 = b"\x03" * 16
    q = ChangeQueue(ME, lambda *a: False, apply_queue_len=100, processing_queue_len=2)
    q.in_flight = 5
    q.recv(full(OTHER, 1))
    q.recv(full(a2, 1))
    q.recv(full(a2, 2))  # drops OTHER's v1, but clears (a2, 1)'s seqs, not (OTHER, 1)
    assert q.dropped == 1
    assert q.seen.get((OTHER, 1)).ranges() == [(0, 0)]
    assert q.seen.get((a2, 1)).ranges() == []
    # so OTHER's dropped v1 is still filtered as seen, while a2's v1 (queued) would pass again
    q.recv(full(OTHER, 1))
    assert [bytes(c.actor_id) for c, _, _ in q.queue] == [a2, a2]


def test_seen_cache_trim_keeps_newest():
    q = ChangeQueue(ME, lambda *a: False, apply_queue_len=1000, processing_queue_len=20)
    q.in_flight = 5
    for v in range(1, 26):
        q.recv(full(OTHER, v))
    assert len(q.seen) == 25  # 5 were dropped from the queue (20 max); their entries keep empty seqs
    q.tick()
    assert len(q.seen) == 10 and [k[1] for k in q.seen.keys] == list(range(16, 26))


def test_seqset():
    s = SeqSet()
    s.extend((0, 3))
    s.extend((5, 6))
    s.extend((4, 4))
    assert s.ranges() == [(0, 6)]
    s.remove((2, 3))
    assert s.ranges() == [(0, 1), (4, 6)]
    assert s.contains_all((4, 6)) and not s.contains_all((1, 4)) and s.contains_all((5, 4))
