"""Failure atomicity of corro_process_multiple_changes' buffered-row commit: a failure in
the pool reserve (CORRO_FAULT=bufpool_reserve injects one, as HBM exhaustion would) must leave no
pending pool segment in the bookie -- the bookie's buffered rows and seq bookkeeping are those before
the call, a re-sent piece buffers again, and the versions complete exactly as on a twin engine that
never saw the failed call. A failure after the call's merge poisons the context
(corro_hip.h "Failure atomicity")."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from corrosion_amd import _lib as L
from tests.test_gpu_agent_device import SCHEMA, _bookie_buffers, _run, canon_rows


def _pieces(ids, ords, nver, seed):
    """per (actor, version): a canonical first half and second half of a partial version, and a
    complete version of another number"""
    from oracle.agent import Changeset
    rng = np.random.default_rng(seed)
    first, second, full = [], [], []
    for a, aid in enumerate(ids):
        site = ords[bytes(aid)]
        for v in range(1, nver + 1):
            k = int(rng.integers(4, 12))
            h = k // 2
            ts = int(rng.integers(1, 1 << 30))
            rows = [dict(pk=int(rng.integers(1, 9)), table_cid=int(rng.integers(1, 5)), col_version=int(rng.integers(1, 4)),
                         db_version=v, cl=1, seq=q, site=site, val0=int(rng.integers(0, 100)), val_type=1)
                    for q in range(k)]
            first.append(Changeset(aid, "full", version=v, seqs=(0, h - 1), last_seq=k - 1, ts=ts, rows=rows[:h]))
            second.append(Changeset(aid, "full", version=v, seqs=(h, k - 1), last_seq=k - 1, ts=ts, rows=rows[h:]))
        v = nver + 1
        rows = [dict(pk=int(rng.integers(1, 9)), table_cid=int(rng.integers(1, 5)), col_version=1, db_version=v,
                     cl=1, seq=q, site=site, val0=int(rng.integers(0, 100)), val_type=1) for q in range(3)]
        full.append(Changeset(aid, "full", version=v, seqs=(0, 2), last_seq=2, ts=7, rows=rows))
    return first, second, full


def _side(ids):
    import corrosion_amd as ca
    eng = ca.MergeEngine(SCHEMA, capacity_hint=1 << 12)
    o = eng.register_sites(ids)
    return eng, ca.agent.Bookie(), {bytes(ids[q]): int(o[q]) for q in range(len(ids))}


def _ready(bk):
    n = C.c_uint64()
    L.check(L.lib().corro_bookie_take_ready(bk._h, None, None, 0, C.byref(n)))
    act = (C.c_uint8 * (16 * max(1, n.value)))()
    ver = (C.c_uint64 * max(1, n.value))()
    L.check(L.lib().corro_bookie_take_ready(bk._h, act, ver, n.value, C.byref(n)))
    return [(bytes(act[16 * k:16 * k + 16]), int(ver[k])) for k in range(n.value)]


def _state(bk, ids, nver):
    return (_bookie_buffers(bk, ids, nver),
            [(bk.last(bytes(a)), bk.needed(bytes(a)), [bk.partial(bytes(a), v) for v in range(1, nver + 2)])
             for a in ids])


def test_failed_pool_reserve_leaves_no_pending_segments(monkeypatch):
    """(device headers: the path whose canonical partial rows stay in the HBM pool)"""
    import corrosion_amd as ca
    device = "headers"
    import synth
    nver = 5
    ids = synth.site_ids(4, 17)
    eng, bk, ords = _side(ids)
    twin, tbk, tords = _side(ids)
    assert ords == tords
    first, second, _full = _pieces(ids, ords, nver, 3)
    # call 1: the first halves land in the device pool on both engines
    assert _run(eng, bk, ords, first, device)[0] == _run(twin, tbk, tords, first, device)[0]
    # call 2 fails in the buffered-row commit (no merge ran: partial pieces only). (The bookie is not
    # read before it: a read brings a key's pool rows to the host, and the call must meet them in HBM.)
    monkeypatch.setenv("CORRO_FAULT", "bufpool_reserve")
    with pytest.raises(ca.CorroError, match="injected fault"):
        _run(eng, bk, ords, second, device)
    monkeypatch.delenv("CORRO_FAULT")
    assert _ready(bk) == []                            # nothing of the failed call completed
    assert _state(bk, ids, nver) == _state(tbk, ids, nver)  # nor is buffered or booked
    # the context is not poisoned (nothing was written) and the re-sent pieces complete the versions
    got = _run(eng, bk, ords, second, device)
    want = _run(twin, tbk, tords, second, device)
    assert got == want
    assert _state(bk, ids, nver) == _state(tbk, ids, nver)
    for e, b in ((eng, bk), (twin, tbk)):
        rd = _ready(b)
        assert len(rd) == len(ids) * nver
        for a, v in rd:
            r = C.c_int()
            L.check(L.lib().corro_process_fully_buffered(e._h, b._h, a, v, C.byref(r)))
    assert canon_rows(eng.export()) == canon_rows(twin.export())
    assert _state(bk, ids, nver) == _state(tbk, ids, nver)


def test_failure_after_the_merge_poisons_the_context(monkeypatch):
    import corrosion_amd as ca
    import synth
    nver = 3
    ids = synth.site_ids(3, 23)
    eng, bk, ords = _side(ids)
    first, _second, full = _pieces(ids, ords, nver, 5)
    monkeypatch.setenv("CORRO_FAULT", "bufpool_reserve")
    with pytest.raises(ca.CorroError, match="poisoned"):
        _run(eng, bk, ords, full + first, "headers")   # complete versions merge, then the commit fails
    monkeypatch.delenv("CORRO_FAULT")
    assert _bookie_buffers(bk, ids, nver) == {(bytes(a), v): [] for a in ids for v in range(1, nver + 1)}
    with pytest.raises(ca.CorroError, match="poisoned"):
        _run(eng, bk, ords, first, "headers")
    eng.reset()                                        # the caller re-seeds state and bookie
    bk = ca.agent.Bookie()
    _run(eng, bk, ords, full + first, "headers")


def test_failed_merge_leaves_the_bookie_as_it_was():
    """A call large enough that its buffered-row commit is prepared on a host thread alongside the
    merge (>= 4096 host-walked changesets): when the merge fails (a sentinel with a negative
    col_version: CORRO_E_RANGE before anything is written) the call fails as a whole -- the bookie holds
    nothing of it, the context is not poisoned, and the same call without the bad changeset then gives
    what a twin that never saw the failure gives."""
    import corrosion_amd as ca
    import synth
    from oracle.agent import Changeset
    nver = 40
    ids = synth.site_ids(64, 29)
    eng, bk, ords = _side(ids)
    twin, tbk, tords = _side(ids)
    first, second, full = _pieces(ids, ords, nver, 7)
    call = [x for pair in zip(first, second) for x in pair] + full
    assert len(first) + len(second) >= 4096
    aid = ids[0]
    bad = Changeset(aid, "full", version=nver + 2, seqs=(0, 0), last_seq=0, ts=9,
                    rows=[dict(pk=3, table_cid=0, col_version=-1, db_version=nver + 2, cl=1, seq=0,
                               site=ords[bytes(aid)], val0=0, val_type=1)])
    before = _state(bk, ids, nver)
    with pytest.raises(ca.CorroError):
        _run(eng, bk, ords, call + [bad], "headers")
    assert _ready(bk) == []
    assert _state(bk, ids, nver) == before
    assert eng.count() == 0
    got = _run(eng, bk, ords, call, "headers")
    want = _run(twin, tbk, tords, call, "headers")
    assert got == want
    assert _state(bk, ids, nver) == _state(tbk, ids, nver)
    assert sorted(_ready(bk)) == sorted(_ready(tbk))
    assert canon_rows(eng.export()) == canon_rows(twin.export())
