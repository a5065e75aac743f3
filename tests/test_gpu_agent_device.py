"""process_multiple_changes end to end against the CPU restatement (oracle/agent.py, util.rs:691-1037
over the pinned merge fold), with the change batch in device memory (CORRO_MEM_DEVICE: the
drop-in path corro_decode_frames feeds) and in host memory.

Random calls mix, from several actors arriving interleaved: complete versions (conflicting cells,
deletes / resurrects), versions re-sent inside a call and across calls, empty versions, partial
versions completed later, versions arriving with gaps that are filled later, and versions naming
an unknown column (rolled back alone). Checked per call: known outcomes and impactful flags; at the
end: the merged state, crsql_db_versions and every actor's gap bookkeeping. Also: the applied batch
built zero-copy (one contiguous run) and by the gather kernel give the same result.
"""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SCHEMA = {"t": ["a", "b", "c", "d"], "u": ["x", "y"]}
NACT = 5


def _calls(seed, ncalls=6, per_call=40, clean=(), empty_sets=0.0):
    """Random calls; actors in `clean` never re-send, never send partial or Empty versions (each of
    their calls is a run of complete Full versions ascending, gaps and empty Full versions allowed:
    the device-header path decides them without the host)."""
    from oracle.agent import Changeset, UNKNOWN
    rng = np.random.default_rng(seed)
    import synth
    ids = synth.site_ids(NACT, seed)
    rng.shuffle(ids)                                   # ordinal order != ActorId order
    nextv = [1] * NACT
    sent, held = [], []                                # earlier changesets; second halves of partials
    cl_of = {}                                         # (table, pk) -> causal length the actors agree on

    def rows(a, version, k):
        out = []
        for s in range(k):
            t = int(rng.integers(0, 2))
            ncols = 4 if t == 0 else 2
            pk = int(rng.integers(1, 12))
            cl = cl_of.get((t, pk), 1)
            r = rng.random()
            if r < 0.08:                               # delete
                cl = cl + 1 if cl % 2 else cl
                cl_of[(t, pk)] = cl
                out.append(dict(pk=pk, table_cid=t << 16, col_version=cl, db_version=version, cl=cl, seq=s,
                                site=a, val0=0, val_type=5))
                continue
            if r < 0.14 or cl % 2 == 0:                # pk-only resurrect / insert
                cl = cl + 1 if cl % 2 == 0 else cl
                cl_of[(t, pk)] = cl
                out.append(dict(pk=pk, table_cid=t << 16, col_version=cl, db_version=version, cl=cl, seq=s,
                                site=a, val0=0, val_type=5))
                continue
            out.append(dict(pk=pk, table_cid=(t << 16) | int(rng.integers(1, ncols + 1)),
                            col_version=int(rng.integers(1, 4)), db_version=version, cl=cl, seq=s, site=a,
                            val0=int(rng.integers(0, 5)), val_type=1))
        return out

    calls = []
    for _c in range(ncalls):
        call = list(held)
        held = []
        for _k in range(per_call):
            a = int(rng.integers(0, NACT))
            r = rng.random()
            if a in clean:
                if rng.random() < 0.1:
                    nextv[a] += int(rng.integers(1, 3))
                v = nextv[a]
                nextv[a] += 1
                k = 0 if rng.random() < 0.05 else int(rng.integers(1, 9))
                rr = rows(a, v, k)
                if k and rng.random() < 0.06:
                    rr[int(rng.integers(0, k))]["table_cid"] = UNKNOWN
                cs = Changeset(ids[a], "full", version=v, seqs=(0, max(k - 1, 0)), last_seq=max(k - 1, 0),
                               ts=int(rng.integers(1, 1 << 40)), rows=rr)
                call.append(cs)
                sent.append(cs)
                continue
            if r < 0.12 and sent:                      # re-sent (same call or an earlier one)
                call.append(sent[int(rng.integers(0, len(sent)))])
                continue
            if rng.random() < 0.1:
                nextv[a] += int(rng.integers(1, 3))    # leave a gap (never filled: stays needed)
            v = nextv[a]
            nextv[a] += 1
            if r < 0.2:
                n = int(rng.integers(1, 3))
                cs = Changeset(ids[a], "empty", versions=(v, v + n - 1))
                nextv[a] += n - 1
            else:
                k = int(rng.integers(1, 9))
                rr = rows(a, v, k)
                ts = int(rng.integers(1, 1 << 40))
                if r < 0.26:                           # an unknown column in the version
                    rr[int(rng.integers(0, k))]["table_cid"] = UNKNOWN
                if r > 0.9 and k >= 2:                 # partial: first half now, rest next call
                    h = k // 2
                    cs = Changeset(ids[a], "full", version=v, seqs=(0, h - 1), last_seq=k - 1, ts=ts, rows=rr[:h])
                    held.append(Changeset(ids[a], "full", version=v, seqs=(h, k - 1), last_seq=k - 1, ts=ts,
                                          rows=rr[h:]))
                else:
                    cs = Changeset(ids[a], "full", version=v, seqs=(0, k - 1), last_seq=k - 1, ts=ts, rows=rr)
            call.append(cs)
            sent.append(cs)
        calls.append(call)
    if held:
        calls.append(held)
    if empty_sets:  # Changeset::EmptySet from random actors, at random places (own rng: seeds keep their calls)
        erng = np.random.default_rng(seed + 1000)
        for call in calls:
            for _k in range(int(erng.binomial(len(call), empty_sets))):
                a = int(erng.integers(0, NACT))
                v0 = int(erng.integers(1, 50))
                cs = Changeset(ids[a], "empty_set", versions=[(v0, v0 + int(erng.integers(0, 4)))],
                               ts=int(erng.integers(1, 1 << 40)))
                call.insert(int(erng.integers(0, len(call) + 1)), cs)
    return ids, calls


FIELDS = {"pk": np.uint64, "table_cid": np.uint32, "col_version": np.int64, "db_version": np.int64,
          "cl": np.uint32, "seq": np.uint32, "site": np.uint32, "val0": np.uint64, "val_type": np.uint8,
          "ts": np.uint64}


def _run(eng, bk, ordinal, call, device, order=None, drop=()):
    """corro_process_multiple_changes on one call; the batch laid out in `order` of the changesets
    (default: arrival order). device: False (host batch), True (device batch) or "headers" (device
    batch, headers and known: CORRO_MEM_DEVICE_HEADERS). Returns (known list, impactful per
    changeset). drop: batch fields left out (val_type: an INTEGER-only batch, every column value here
    is INTEGER and a sentinel's value is not stored; ts: the changesets' ts only)."""
    import torch
    from corrosion_amd import _lib as L
    order = list(range(len(call))) if order is None else order
    off, rows = {}, []
    for i in order:
        off[i] = len(rows)
        rows.extend(dict(r, ts=call[i].ts) for r in call[i].rows)
    n = len(rows)
    arr = {k: np.array([r[k] for r in rows] or [0], dt) for k, dt in FIELDS.items() if k not in drop}
    keep = []
    s = L.Changes()
    s.n = n
    for k, a in arr.items():
        if device:
            t = torch.from_numpy(a.view({8: np.int64, 4: np.int32, 1: np.uint8}[a.itemsize])).cuda()
            keep.append(t)
            setattr(s, k, t.data_ptr())
        else:
            keep.append(a)
            setattr(s, k, a.ctypes.data)
    descs = (L.Changeset * max(1, len(call)))()
    abufs = []
    for i, c in enumerate(call):
        d = descs[i]
        ab = C.create_string_buffer(bytes(c.actor), 16)
        abufs.append(ab)
        d.actor_id = C.addressof(ab)
        d.site = ordinal[bytes(c.actor)]
        d.ts = c.ts
        if c.kind == "full":
            d.kind = L.CORRO_CS_FULL
            d.version_start = d.version_end = c.version
            d.seq_start, d.seq_end = c.seqs
            d.last_seq = c.last_seq
            d.change_off, d.change_count = off[i], len(c.rows)
        elif c.kind == "empty":
            d.kind = L.CORRO_CS_EMPTY
            d.version_start, d.version_end = c.versions
        else:
            d.kind = L.CORRO_CS_EMPTY_SET  # (its ranges travel beside the header; unused by the apply)
    known = np.zeros(max(1, len(call)), np.int32)
    if device:
        imp = torch.zeros(max(n, 1), dtype=torch.uint8, device="cuda")
        ip = imp.data_ptr()
        torch.cuda.synchronize()
    else:
        imp = np.zeros(max(n, 1), np.uint8)
        ip = imp.ctypes.data
    out = L.ProcessOut()
    out.known, out.impactful = known.ctypes.data, ip
    mem = L.CORRO_MEM_DEVICE if device else L.CORRO_MEM_HOST
    cs_arg = descs
    if device == "headers":
        raw = np.frombuffer(bytes(descs), np.uint8)
        dcs = torch.from_numpy(raw.copy()).cuda()
        dknown = torch.full((max(1, len(call)),), -99, dtype=torch.int32, device="cuda")
        keep += [dcs, dknown]
        torch.cuda.synchronize()
        cs_arg, out.known, mem = C.c_void_p(dcs.data_ptr()), dknown.data_ptr(), L.CORRO_MEM_DEVICE_HEADERS
    L.check(L.lib().corro_process_multiple_changes(eng._h, bk._h, cs_arg, len(call), C.byref(s), mem, C.byref(out)))
    if device == "headers":
        known = dknown.cpu().numpy()
    imp = imp.cpu().numpy() if device else imp
    kn = [L.KNOWN.get(int(k), int(k)) for k in known[:len(call)]]
    return kn, [list(imp[off[i]:off[i] + len(c.rows)]) if c.kind == "full" else [] for i, c in enumerate(call)]


def canon_rows(rows):
    keys = ("table_cid", "pk", "val_type", "val0", "col_version", "db_version", "site", "cl", "seq", "ts")
    return sorted(zip(*[np.asarray(rows[k]).tolist() for k in keys]))


def _overlap_calls(seed, ncalls=5, per_call=60, base=0):
    """Adversarial calls for the per-changeset device decisions: versions from a small window per
    actor (base + 0..14 or 0..39, a window near 2^40 with base), so ranges overlap all the time -- complete
    and partial Full versions, Empty ranges crossing each other and Full versions, exact duplicates
    (same and different content), EmptySet, version 0 -- in random arrival order, over calls that move
    each actor's booked max."""
    from oracle.agent import Changeset
    rng = np.random.default_rng(seed)
    import synth
    ids = synth.site_ids(NACT, seed)
    calls, prev = [], []
    win = 15 if seed % 2 else 40
    for c in range(ncalls):
        call = []
        lo = base + 3 * c                                 # the window climbs: some versions go below max
        for _k in range(per_call):
            a = int(rng.integers(0, NACT))
            v = lo + int(rng.integers(0, win))
            r = rng.random()
            if r < 0.08 and prev:
                call.append(prev[int(rng.integers(0, len(prev)))])
                continue
            if r < 0.12:
                cs = Changeset(ids[a], "empty_set", versions=[(v, v + 1)], ts=int(rng.integers(1, 1 << 30)))
            elif r < 0.3:
                vs = int(rng.integers(0, 2)) * v if base == 0 else v  # (ranges from 0 too)
                cs = Changeset(ids[a], "empty", versions=(vs, v + int(rng.integers(0, 4))))
            else:
                if base == 0 and rng.random() < 0.03:
                    v = 0
                k = int(rng.integers(0, 5))
                rr = [dict(pk=int(rng.integers(1, 6)), table_cid=(0 << 16) | int(rng.integers(1, 5)),
                           col_version=int(rng.integers(1, 4)), db_version=v, cl=1, seq=s, site=a,
                           val0=int(rng.integers(0, 4)), val_type=1) for s in range(k)]
                ts = int(rng.integers(1, 1 << 30))
                if k >= 2 and rng.random() < 0.25:       # a partial (some halves never arrive)
                    h = k // 2
                    part = (rr[:h], (0, h - 1)) if rng.random() < 0.5 else (rr[h:], (h, k - 1))
                    cs = Changeset(ids[a], "full", version=v, seqs=part[1], last_seq=k - 1, ts=ts, rows=part[0])
                else:
                    cs = Changeset(ids[a], "full", version=v, seqs=(0, max(k - 1, 0)), last_seq=max(k - 1, 0),
                                   ts=ts, rows=rr)
            call.append(cs)
            if rng.random() < 0.1:
                call.append(cs)                           # an exact duplicate in the same call
        prev = list(call)
        calls.append(call)
    return ids, calls


def _check_against_oracle(seed, device, order_fn=None, clean=(), empty_sets=0.0, calls_fn=None, drop=()):
    import corrosion_amd as ca
    from oracle.agent import AgentOracle
    ids, calls = calls_fn(seed) if calls_fn else _calls(seed, clean=clean, empty_sets=empty_sets)
    if empty_sets:
        assert any(c.kind == "empty_set" for call in calls for c in call)
    eng = ca.MergeEngine(SCHEMA, capacity_hint=1 << 12)
    ords = eng.register_sites(ids)
    ordinal = {bytes(ids[k]): int(ords[k]) for k in range(NACT)}
    bk = ca.agent.Bookie()
    ref = AgentOracle(ids)
    for call in calls:
        for c in call:                       # oracle rows name sites by ordinal too
            for r in c.rows:
                r["site"] = ordinal[bytes(c.actor)]
        order = order_fn(call) if order_fn else None
        got_known, got_imp = _run(eng, bk, ordinal, call, device, order, drop)
        exp_known, exp_imp = ref.process(call)
        assert got_known == exp_known
        assert got_imp == exp_imp
    assert canon_rows(eng.export()) == canon_rows(ref.export())
    dbv = list(ref.fold.db_versions())
    for a, v in ref.set_dbv.items():
        o = ordinal[a]
        dbv[o] = max(dbv[o], v)
    assert list(eng.db_versions()) == dbv
    for a in ordinal:
        assert bk.last(a) == ref.last(a)
        assert bk.needed(a) == ref.needed(a)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_device_batch_matches_restatement(seed):
    _check_against_oracle(seed, device=True)


@pytest.mark.parametrize("device", [True, "headers"])
@pytest.mark.parametrize("drop", [("val_type",), ("ts",), ("val_type", "ts")])
def test_integer_batch_and_changeset_ts_match_restatement(drop, device):
    # the ts routes of the apply: an INTEGER-only batch stages each change's ts in its record (by
    # input index, or by application position when only the changesets carry one); a batch with
    # value words keeps the per-position ts array
    _check_against_oracle(4, device=device, drop=drop)


@pytest.mark.parametrize("seed", [7, 8])
def test_device_batch_gather_path_matches_restatement(seed, monkeypatch):
    """the applied batch gathered into application order (the path for inputs that are not one
    aligned apply chunk) instead of staged in place with application positions"""
    monkeypatch.setenv("CORRO_AGENT_GATHER", "1")
    _check_against_oracle(seed, device=True)


@pytest.mark.parametrize("seed", [4, 5])
def test_host_batch_matches_restatement(seed):
    _check_against_oracle(seed, device=False)


def test_batch_in_application_order_zero_copy():
    """The batch laid out in application order (actors by id, arrival order within): the applied
    changesets are one contiguous run, so the engine merges the caller's arrays in place."""
    def app_order(call):
        return sorted(range(len(call)), key=lambda i: (bytes(call[i].actor), i))
    _check_against_oracle(6, device=True, order_fn=app_order)


@pytest.mark.parametrize("seed", [1, 2])
def test_device_headers_matches_restatement(seed):
    """CORRO_MEM_DEVICE_HEADERS: headers and known on the device; every actor slow here (re-sends,
    partials, Empty versions), so the host walks the fetched headers"""
    _check_against_oracle(seed, device="headers")


@pytest.mark.parametrize("seed,clean", [(11, (0, 1, 2)), (12, (0, 1, 2, 3, 4)), (13, (1, 3))])
def test_device_headers_fast_actors_match_restatement(seed, clean):
    """actors decided on the device (complete Full versions ascending, gaps, empty Full versions,
    unknown names) next to slow ones, in one call"""
    _check_against_oracle(seed, device="headers", clean=clean)


@pytest.mark.parametrize("device,clean", [(True, ()), (False, ()), ("headers", ()), ("headers", (0, 1, 2))])
def test_empty_set_changesets_match_restatement(device, clean):
    """Changeset::EmptySet (broadcast.rs:114-148) mixed into random calls: its versions() is the dummy
    0..=0 (:176), which contains_all always holds, so process_multiple_changes skips it in pass 1
    (util.rs:724-733): known = skipped, no crsql_set_db_version, no gap rows -- on every header path,
    next to fast and slow actors"""
    _check_against_oracle(21, device=device, clean=clean, empty_sets=0.1)


@pytest.mark.parametrize("seed", [31, 32, 33])
@pytest.mark.parametrize("device", ["headers", True])
def test_overlapping_versions_match_restatement(seed, device):
    """The per-changeset device decisions next to the host walk: only changesets no other changeset of
    their actor overlaps, above the booked max, are decided on the device; everything else (overlaps,
    duplicates with other content, partials, ranges from version 0) must come out as the reference's
    per-actor passes say -- on the device-header path and the host-header one"""
    _check_against_oracle(seed, device=device, calls_fn=_overlap_calls)


def test_overlapping_versions_near_2_40_match_restatement():
    """versions at and above 2^40 - 1 share the decision sort's key: they always go to the host walk"""
    _check_against_oracle(34, device="headers", calls_fn=lambda s: _overlap_calls(s, base=(1 << 40) - 9))


def test_device_headers_fast_gather_path(monkeypatch):
    monkeypatch.setenv("CORRO_AGENT_GATHER", "1")
    _check_against_oracle(14, device="headers", clean=(0, 2, 4))


def _dev_call(eng, bk, descs, n_cs, batch_arrays, n):
    """corro_process_multiple_changes with CORRO_MEM_DEVICE_HEADERS on raw descriptors; returns
    (rc, known list)."""
    import torch
    from corrosion_amd import _lib as L
    s = L.Changes()
    s.n = n
    keep = []
    for k, a in batch_arrays.items():
        t = torch.from_numpy(a.view({8: np.int64, 4: np.int32, 1: np.uint8}[a.itemsize])).cuda()
        keep.append(t)
        setattr(s, k, t.data_ptr())
    dcs = torch.from_numpy(np.frombuffer(bytes(descs), np.uint8).copy()).cuda()
    dknown = torch.full((max(1, n_cs),), 77, dtype=torch.int32, device="cuda")
    out = L.ProcessOut()
    out.known = dknown.data_ptr()
    torch.cuda.synchronize()
    rc = L.lib().corro_process_multiple_changes(eng._h, bk._h, C.c_void_p(dcs.data_ptr()), n_cs, C.byref(s),
                                                L.CORRO_MEM_DEVICE_HEADERS, C.byref(out))
    return rc, dknown[:n_cs].cpu().tolist()


def _one_full_batch(site, version, k, pk0=1):
    rows = [dict(pk=pk0 + j, table_cid=(0 << 16) | 1, col_version=1, db_version=version, cl=1, seq=j, site=site,
                 val0=j, val_type=1, ts=5) for j in range(k)]
    return {key: np.array([r[key] for r in rows], dt) for key, dt in FIELDS.items()}


def test_device_headers_bad_span_and_site_fail_untouched():
    """A span outside the batch or an unregistered site ordinal fails the call before anything is
    decided: every outcome Skipped, no state, no bookkeeping (the host-header path's errors)."""
    import corrosion_amd as ca
    from corrosion_amd import _lib as L
    import synth
    ids = synth.site_ids(2, 5)
    eng = ca.MergeEngine(SCHEMA, capacity_hint=1 << 10)
    ords = eng.register_sites(ids)
    bk = ca.agent.Bookie()
    arrs = _one_full_batch(int(ords[0]), 1, 4)
    for bad in ("span", "site"):
        descs = (L.Changeset * 2)()
        for i in range(2):
            d = descs[i]
            d.site, d.kind = int(ords[0]), L.CORRO_CS_FULL
            d.version_start = d.version_end = i + 1
            d.seq_start, d.seq_end, d.last_seq = 0, 1, 1
            d.change_off, d.change_count = 2 * i, 2
        if bad == "span":
            descs[1].change_count = 3          # [2, 5) is outside the 4-change batch
        else:
            descs[1].site = 99                 # not a registered ordinal
        rc, known = _dev_call(eng, bk, descs, 2, arrs, 4)
        assert rc == -1                       # CORRO_E_INVALID
        assert known == [0, 0]
        assert eng.count() == 0
        assert bk.last(bytes(ids[0])) is None


def test_device_headers_empty_and_zero_calls():
    """No changesets at all, and a call of only empty Full versions (no changes): the latter bump
    crsql_db_versions and the bookkeeping, merge nothing."""
    import corrosion_amd as ca
    from corrosion_amd import _lib as L
    import synth
    ids = synth.site_ids(2, 6)
    eng = ca.MergeEngine(SCHEMA, capacity_hint=1 << 10)
    ords = eng.register_sites(ids)
    bk = ca.agent.Bookie()
    arrs = _one_full_batch(int(ords[1]), 1, 1)
    rc, known = _dev_call(eng, bk, (L.Changeset * 1)(), 0, arrs, 1)
    assert rc == 0 and known == []
    descs = (L.Changeset * 3)()
    for i in range(3):
        d = descs[i]
        d.site, d.kind = int(ords[1]), L.CORRO_CS_FULL
        d.version_start = d.version_end = i + 1
        d.seq_start = d.seq_end = d.last_seq = 0
        d.change_off, d.change_count = 0, 0
    rc, known = _dev_call(eng, bk, descs, 3, arrs, 1)
    assert rc == 0
    assert known == [2, 2, 2]                  # Cleared (process_empty_version)
    assert eng.count() == 0
    assert bk.last(bytes(ids[1])) == 3 and bk.needed(bytes(ids[1])) == []
    assert list(eng.db_versions())[int(ords[1])] == 3


@pytest.mark.parametrize("seed,clean", [(21, ()), (22, (0, 1, 2, 3, 4)), (23, (1, 2))])
def test_host_headers_staged_to_device_match_restatement(seed, clean, monkeypatch):
    """CORRO_MEM_DEVICE with host headers staged through the device header passes (the path large
    calls take; forced here): same outcomes, flags, state and bookkeeping as the restatement"""
    monkeypatch.setenv("CORRO_AGENT_STAGE_HEADERS", "1")
    _check_against_oracle(seed, device=True, clean=clean)


def _buffer_calls(seed, nact=3, nver=6, ncalls=5):
    """Partial versions sent in overlapping pieces across calls: re-sent seqs carry different
    contents (the stored row must win), some pieces are non-canonical (rows out of seq order, or a
    row missing), some versions arrive complete."""
    from oracle.agent import Changeset
    rng = np.random.default_rng(seed)
    import synth
    ids = synth.site_ids(nact, seed)
    pieces = []
    for a in range(nact):
        for v in range(1, nver + 1):
            k = int(rng.integers(3, 11))
            ts = int(rng.integers(1, 1 << 30))

            def rows(s, e, a=a, v=v):
                return [dict(pk=int(rng.integers(1, 7)), table_cid=(0 << 16) | int(rng.integers(1, 5)),
                             col_version=int(rng.integers(1, 4)), db_version=v, cl=1, seq=q, site=a,
                             val0=int(rng.integers(0, 1000)), val_type=1) for q in range(s, e + 1)]
            if rng.random() < 0.15:
                pieces.append(Changeset(ids[a], "full", version=v, seqs=(0, k - 1), last_seq=k - 1, ts=ts,
                                        rows=rows(0, k - 1)))
                continue
            for _p in range(int(rng.integers(2, 5))):
                s = int(rng.integers(0, k))
                e = int(rng.integers(s, k))
                rr = rows(s, e)
                r = rng.random()
                if r < 0.15 and len(rr) > 1:
                    rr = rr[::-1]                      # out of seq order
                elif r < 0.25 and len(rr) > 1:
                    rr = rr[:-1]                       # a row short of the seq range
                pieces.append(Changeset(ids[a], "full", version=v, seqs=(s, e), last_seq=k - 1, ts=ts, rows=rr))
            pieces.append(Changeset(ids[a], "full", version=v, seqs=(0, k - 1), last_seq=k - 1, ts=ts,
                                    rows=rows(0, k - 1)) if rng.random() < 0.1 else
                          Changeset(ids[a], "full", version=v, seqs=(0, 0), last_seq=k - 1, ts=ts, rows=rows(0, 0)))
    order = rng.permutation(len(pieces))
    calls = [[] for _ in range(ncalls)]
    for j in order:
        calls[int(rng.integers(0, ncalls))].append(pieces[j])
    return ids, calls


def _bookie_buffers(bk, ids, nver):
    from corrosion_amd import serve
    out = {}
    for a in ids:
        for v in range(1, nver + 1):
            rows, n = serve._buffered_rows(bk, bytes(a), v, 0, (1 << 32) - 1)
            out[(bytes(a), v)] = sorted(zip(*[rows[k][:n].tolist() for k in sorted(rows)]))
    return out


@pytest.mark.parametrize("seed", [41, 42, 43])
def test_device_buffered_rows_match_host_path(seed):
    """Partial changesets of a device-header call keep their rows in HBM (bufpool.hip): pieces re-sent
    with other contents (ON CONFLICT DO NOTHING: the stored row wins), non-canonical pieces next to
    canonical ones of the same version (the key goes to the host), buffered rows read back, and
    process_fully_buffered_changes of every ready version -- outcomes, buffered rows, committed
    counts, merged state and bookkeeping equal to the host-memory path's"""
    import corrosion_amd as ca
    from corrosion_amd import _lib as L
    nver = 6
    ids, calls = _buffer_calls(seed, nver=nver)
    sides = []
    for _k in range(2):
        eng = ca.MergeEngine(SCHEMA, capacity_hint=1 << 12)
        ords = eng.register_sites(ids)
        sides.append((eng, ca.agent.Bookie(), {bytes(ids[q]): int(ords[q]) for q in range(len(ids))}))
    for c in (c for call in calls for c in call):
        for r in c.rows:
            r["site"] = sides[0][2][bytes(c.actor)]
    assert sides[0][2] == sides[1][2]

    def ready(bk):
        n = C.c_uint64()
        L.check(L.lib().corro_bookie_take_ready(bk._h, None, None, 0, C.byref(n)))
        act = (C.c_uint8 * (16 * max(1, n.value)))()
        ver = (C.c_uint64 * max(1, n.value))()
        L.check(L.lib().corro_bookie_take_ready(bk._h, act, ver, n.value, C.byref(n)))
        return [(bytes(act[16 * k:16 * k + 16]), int(ver[k])) for k in range(n.value)]

    for ci, call in enumerate(calls):
        got = [_run(eng, bk, o, call, dev)[0] for (eng, bk, o), dev in zip(sides, ("headers", False))]
        assert got[0] == got[1]
        if ci == 2:   # a read in the middle: device keys come to the host, later pieces mix with them
            assert _bookie_buffers(sides[0][1], ids, nver) == _bookie_buffers(sides[1][1], ids, nver)
        rd = [ready(bk) for _e, bk, _o in sides]
        assert rd[0] == rd[1]
        for a, v in rd[0]:
            imp = []
            for eng, bk, _o in sides:
                r = C.c_int()
                L.check(L.lib().corro_process_fully_buffered(eng._h, bk._h, a, v, C.byref(r)))
                imp.append(r.value)
            assert imp[0] == imp[1]
    assert _bookie_buffers(sides[0][1], ids, nver) == _bookie_buffers(sides[1][1], ids, nver)
    (ea, ba, _), (eb, bb, _) = sides
    assert canon_rows(ea.export()) == canon_rows(eb.export())
    assert list(ea.db_versions()) == list(eb.db_versions())
    assert ea.committed("t") == eb.committed("t")
    for a in ids:
        assert ba.last(bytes(a)) == bb.last(bytes(a))
        assert ba.needed(bytes(a)) == bb.needed(bytes(a))
        for v in range(1, nver + 1):
            assert ba.partial(bytes(a), v) == bb.partial(bytes(a), v)


def _mixed_scale_calls(seed, nact=64, nver=120, per=8, ncalls=3):
    """agent_e2e_mixed's shape at a test size: versions arriving round-robin across actors, ~10 %
    re-sent later in the call, ~5 % as two partial halves (the second half later), ~5 % Empty, over
    calls whose versions continue (each call's versions above the previous call's)."""
    from oracle.agent import Changeset
    rng = np.random.default_rng(seed)
    import synth
    ids = synth.site_ids(nact, seed)
    calls, v0 = [], 0
    for _c in range(ncalls):
        head, tail = [], []
        for v in range(v0 + 1, v0 + nver + 1):
            for a in range(nact):
                rr = [dict(pk=int(rng.integers(1, 4000)), table_cid=(0 << 16) | int(rng.integers(1, 5)),
                           col_version=int(rng.integers(1, 6)), db_version=v, cl=1, seq=q, site=a,
                           val0=int(rng.integers(0, 1 << 40)), val_type=1) for q in range(per)]
                ts = int(rng.integers(1, 1 << 40))
                u = rng.random()
                if u < 0.05:
                    cs = Changeset(ids[a], "empty", versions=(v, v))
                elif u < 0.10:
                    h = per // 2
                    cs = Changeset(ids[a], "full", version=v, seqs=(0, h - 1), last_seq=per - 1, ts=ts, rows=rr[:h])
                    tail.append(Changeset(ids[a], "full", version=v, seqs=(h, per - 1), last_seq=per - 1, ts=ts,
                                          rows=rr[h:]))
                else:
                    cs = Changeset(ids[a], "full", version=v, seqs=(0, per - 1), last_seq=per - 1, ts=ts, rows=rr)
                    if rng.random() < 0.10:
                        tail.append(cs)
                head.append(cs)
        order = rng.permutation(len(tail))
        call = list(head)
        for j in order:   # re-sends and second halves into the back half of the call
            call.insert(int(rng.integers(len(call) // 2, len(call) + 1)), tail[j])
        calls.append(call)
        v0 += nver
    return ids, calls


@pytest.mark.parametrize("prep_min", [None, "0"])
def test_mixed_call_at_scale_matches_host_path(prep_min, monkeypatch):
    """The mixed drop-in call at ~8.7 K changesets x 3 calls: device-resident headers (per-changeset
    device decisions, host walk of the rest, partial rows in the device pool) against the
    host-memory path -- outcomes, impactful flags, merged state, db_versions, committed counts, gap
    bookkeeping and partials. prep_min "0": the commit's read-only parts (buffered-row groups, seq-book
    moves, the buffered-meta keys the commit leaves) on the preparation thread alongside the merge, as
    calls of 4096 host changesets or more take them (CORRO_AGENT_PREP_MIN)."""
    import corrosion_amd as ca
    if prep_min is not None:
        monkeypatch.setenv("CORRO_AGENT_PREP_MIN", prep_min)
    ids, calls = _mixed_scale_calls(51)
    sides = []
    for _k in range(2):
        eng = ca.MergeEngine(SCHEMA, capacity_hint=1 << 18)
        ords = eng.register_sites(ids)
        sides.append((eng, ca.agent.Bookie(), {bytes(ids[q]): int(ords[q]) for q in range(len(ids))}))
    assert sides[0][2] == sides[1][2]
    for c in (c for call in calls for c in call):
        for r in c.rows:
            r["site"] = sides[0][2][bytes(c.actor)]
    for call in calls:
        got = [_run(eng, bk, o, call, dev) for (eng, bk, o), dev in zip(sides, ("headers", False))]
        assert got[0][0] == got[1][0]
        assert got[0][1] == got[1][1]
        assert "partial" in got[0][0] and "skipped" in got[0][0] and "cleared" in got[0][0]
    (ea, ba, _), (eb, bb, _) = sides
    assert canon_rows(ea.export()) == canon_rows(eb.export())
    assert list(ea.db_versions()) == list(eb.db_versions())
    assert ea.committed("t") == eb.committed("t")
    for a in ids:
        assert ba.last(bytes(a)) == bb.last(bytes(a))
        assert ba.needed(bytes(a)) == bb.needed(bytes(a))


@pytest.mark.parametrize("device,seed,clean", [("headers", 1, ()), ("headers", 12, (0, 1, 2, 3, 4)), (True, 2, ()),
                                               (False, 4, ())])
def test_batched_gap_bookkeeping_route_matches_restatement(device, seed, clean, monkeypatch):
    """Calls with many actors take the batched device gap pass (corro_booked_insert_db_batch) instead
    of the per-actor host insert_db; forced here on small calls: the same outcomes, bookkeeping and
    partials as the restatement, on every header path"""
    monkeypatch.setenv("CORRO_AGENT_GAPS_BATCH", "1")
    _check_against_oracle(seed, device=device, clean=clean)


def test_batched_gap_bookkeeping_route_overlaps_and_buffers(monkeypatch):
    monkeypatch.setenv("CORRO_AGENT_GAPS_BATCH", "1")
    _check_against_oracle(31, device="headers", calls_fn=_overlap_calls)
    test_device_buffered_rows_match_host_path(42)
