"""Batched gap bookkeeping on the device (corro_booked_insert_db_batch, csrc/gaps.hip) against the
reference's own insert_db steps (agent.rs:1605-1868, tests/golden/gaps_kats.json), the host C++
Booked (KAT-pinned: removed / inserted rows) and the oracle's restatement (needed gaps, max)."""
import numpy as np
import pytest

import corrosion_amd as ca
from corrosion_amd.bookkeeping import canonical_ranges, insert_db_batch
from oracle import oracle as O
from tests._util import load_golden

pytestmark = pytest.mark.gpu


def _engine():
    return ca.MergeEngine({"t": ["a"]}, capacity_hint=1024)


def test_gap_kats_batched():
    """The 18 steps of test_booked_insert_db, each step one batched call for one actor carrying the
    previous step's gaps and max."""
    e = _engine()
    steps = load_golden("gaps_kats.json")["steps"]
    gaps, mx, allv = [], None, []
    for st in steps:
        if st.get("reset"):
            gaps, mx, allv = [], None, []
            continue
        (mx, _rm, _ins, gaps, status), = insert_db_batch(e, [mx], [gaps], [st["insert"]])
        assert status == 0
        allv += st["insert"]
        if st["gaps"] is not None:
            assert gaps == [tuple(g) for g in st["gaps"]]
        assert mx == max(r[1] for r in allv)


def _random_state(rng):
    """A Booked state reached by a few random insert_db calls (host C++), and the next call's ranges."""
    b = ca.BookedVersions()
    hist = []
    for _ in range(int(rng.integers(0, 4))):
        k = int(rng.integers(1, 5))
        st = rng.integers(1, 300, size=k)
        hist.append([(int(s), int(s + rng.integers(0, 12))) for s in st])
        b.insert_db(hist[-1])
    k = int(rng.integers(0, 6))
    st = rng.integers(1, 400, size=k)
    nxt = [(int(s), int(s + rng.integers(0, 30))) for s in st]
    return b, hist, nxt


def test_random_actors_vs_host_and_oracle():
    rng = np.random.default_rng(31)
    e = _engine()
    n = 6000
    states = [_random_state(rng) for _ in range(n)]
    got = insert_db_batch(e, [b.last() for b, _, _ in states], [b.needed() for b, _, _ in states],
                          [nxt for _, _, nxt in states])
    for (b, hist, nxt), (mx, rm, ins, gaps, status) in zip(states, got):
        assert status == 0
        rm_h, ins_h = b.insert_db(canonical_ranges(nxt)) if nxt else ([], [])
        assert sorted(rm) == sorted(set(rm_h))          # DELETE rows: a HashSet in the reference
        assert ins == ins_h                              # INSERT rows: RangeInclusiveSet order
        assert gaps == b.needed()
        assert mx == b.last()
        f = O.Booked()
        for h in hist + ([nxt] if nxt else []):
            f.insert_db(h)
        assert gaps == f.needed() and mx == f.max()


def test_non_canonical_input_flagged():
    e = _engine()
    (mx, rm, ins, gaps, status), = insert_db_batch(e, [10], [[(3, 5), (4, 8)]], [[(12, 12)]])
    assert status == -1


def _long_state(rng):
    """An actor with many gaps (a wave each in k_gaps_wave): every other version range applied, then
    the next call's ranges, some spanning many gaps, some above max."""
    b = ca.BookedVersions()
    ng = int(rng.integers(20, 400))
    hist = [[(int(3 * k + 1), int(3 * k + 1)) for k in range(ng)]]
    b.insert_db(hist[0])
    top = 3 * ng + 1
    k = int(rng.integers(0, 90))
    st = rng.integers(1, top + 60, size=k)
    nxt = [(int(s), int(s + rng.integers(0, rng.choice([2, 8, 40])))) for s in st]
    return b, hist, nxt


def test_long_actors_vs_host_and_oracle():
    rng = np.random.default_rng(32)
    e = _engine()
    states = [_long_state(rng) if i % 3 else _random_state(rng) for i in range(3000)]
    got = insert_db_batch(e, [b.last() for b, _, _ in states], [b.needed() for b, _, _ in states],
                          [nxt for _, _, nxt in states])
    nlong = 0
    for (b, hist, nxt), (mx, rm, ins, gaps, status) in zip(states, got):
        nlong += len(b.needed()) + len(canonical_ranges(nxt) if nxt else []) > 32
        assert status == 0
        rm_h, ins_h = b.insert_db(canonical_ranges(nxt)) if nxt else ([], [])
        assert sorted(rm) == sorted(set(rm_h))
        assert ins == ins_h
        assert gaps == b.needed()
        assert mx == b.last()
        f = O.Booked()
        for h in hist + ([nxt] if nxt else []):
            f.insert_db(h)
        assert gaps == f.needed() and mx == f.max()
    assert nlong > 1000


def test_non_canonical_long_actor_flagged():
    e = _engine()
    gaps = [(3 * k + 2, 3 * k + 3) for k in range(50)] + [(150, 151)]   # (149, 150) and (150, 151) overlap
    (mx, rm, ins, gaps_out, status), = insert_db_batch(e, [400], [gaps], [[(402, 402)]])
    assert status == -1
