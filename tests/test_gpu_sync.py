"""GPU parity of the batched need diff (k_needs via corro_compute_needs) against the oracle and
the reference's own test_compute_available_needs assertions (sync.rs:386-500)."""
import numpy as np
import pytest

from oracle import oracle as O
from tests._util import load_golden
from tests.sync_util import decode_needs, entries_from_pairs, kat_expect

pytestmark = pytest.mark.gpu
SYNC = load_golden("sync_kats.json")


def _engine():
    import corrosion_amd as ca
    return ca.MergeEngine({"t": ["a"]}, capacity_hint=1024)


@pytest.mark.parametrize("case", SYNC["cases"], ids=[c["name"] for c in SYNC["cases"]])
def test_sync_kats_gpu(case):
    e = _engine()
    ent = entries_from_pairs([(case["our"], case["their"])])
    assert decode_needs(e.compute_needs(ent), 1)[0] == kat_expect(case["expect"])


def test_sync_state_api_gpu():
    import corrosion_amd as ca
    e = _engine()
    a1 = b"\x01" * 16
    ours = ca.SyncStateV1(actor_id=b"\x00" * 16, heads={a1: 10}, need={a1: [(2, 5), (7, 7)]},
                          partial_need={a1: {9: [(100, 120), (130, 132)]}})
    theirs = ca.SyncStateV1(actor_id=b"\x02" * 16, heads={a1: 13, b"\x00" * 16: 4},
                            partial_need={a1: {9: [(100, 110), (130, 130)]}})
    got = ours.compute_available_needs(theirs, e)
    assert got == {a1: [ca.Full(2, 5), ca.Full(7, 7), ca.Partial(9, ((111, 120), (131, 132))), ca.Full(11, 13)]}


def random_side(rng, with_head=True):
    head = int(rng.integers(1, 200))
    need, x = [], 1
    for _ in range(int(rng.poisson(2))):
        s = x + int(rng.integers(1, 30))
        e = s + int(rng.geometric(0.1))
        need.append([s, e])
        x = e + 2
    partials = {}
    for _ in range(int(rng.integers(0, 3))):
        v = int(rng.integers(1, head + 10))
        rs, y = [], int(rng.integers(0, 5))
        for _ in range(int(rng.integers(0, 4))):
            a = y + int(rng.integers(0, 20))
            b = a + int(rng.integers(0, 20))
            rs.append([a, b])
            y = b + 2
        partials[str(v)] = rs
    return {"head": head if with_head else None, "need": need, "partials": partials}


def test_sync_random_vs_oracle():
    rng = np.random.default_rng(5)
    pairs = [(random_side(rng, with_head=rng.random() < 0.9), random_side(rng)) for _ in range(5000)]
    ent = entries_from_pairs(pairs)
    e = _engine()
    got = e.compute_needs(ent)
    exp = O.needs(ent)
    for k in ("need_off", "seq_off", "kind", "start", "end", "sr_off", "sr_n", "s_start", "s_end"):
        assert np.array_equal(got[k], exp[k]), k


def test_sync_device_resident_config4_shape_vs_oracle():
    """Config-4-shaped entries generated in HBM, need diff on device, checked against the oracle."""
    import torch
    import synth
    from corrosion_amd.sync import _needs_device
    ent = synth.sync_entries_torch(3000, 16, 9, device="cuda")
    e = _engine()
    got = _needs_device(e, ent)
    host = {k: v.cpu().numpy() for k, v in ent.items()}
    exp = O.needs(host)
    for k in ("need_off", "seq_off", "kind", "start", "end", "sr_off", "sr_n", "s_start", "s_end"):
        assert np.array_equal(got[k].cpu().numpy().astype(np.uint64), exp[k].astype(np.uint64)), k


def _dense_side(rng, nranges, head):
    need, x = [], 1
    for _ in range(nranges):
        s = x + int(rng.integers(1, 4))
        e = s + int(rng.integers(0, 3))
        need.append([s, e])
        x = e + 2
    return {"head": head, "need": need, "partials": {}}


@pytest.mark.parametrize("dense", ["theirs", "ours", "both"])
def test_sync_lds_caps_exceeded_vs_oracle(dense):
    """Workgroups whose staged need ranges (> 640 per side) or outputs (> 960 needs) exceed the LDS
    caps of k_needs take the global-memory path; mixed with normal workgroups in one launch."""
    rng = np.random.default_rng(11)
    pairs = []
    for i in range(1200):
        heavy = 256 <= i < 768  # two whole workgroups of heavy entries
        nt = 12 if heavy and dense in ("theirs", "both") else int(rng.poisson(2))
        no = 12 if heavy and dense in ("ours", "both") else int(rng.poisson(2))
        their = _dense_side(rng, nt, 300)
        our = _dense_side(rng, no, int(rng.integers(1, 100)))
        pairs.append((our, their))
    ent = entries_from_pairs(pairs)
    e = _engine()
    got = e.compute_needs(ent)
    exp = O.needs(ent)
    for k in ("need_off", "seq_off", "kind", "start", "end", "sr_off", "sr_n", "s_start", "s_end"):
        assert np.array_equal(got[k], exp[k]), k


# ---- one-pass form (corro_compute_needs_onepass: decoupled look-back, inputs read once) ----------

def _to_dev(ent):
    import torch
    return {k: torch.from_numpy(np.ascontiguousarray(v).view(np.int64)).cuda() for k, v in ent.items()}


def _check_1pass(ent_host, exp=None):
    from corrosion_amd.sync import _needs_device_1pass
    got = _needs_device_1pass(_engine(), _to_dev(ent_host))
    exp = O.needs(ent_host) if exp is None else exp
    for k in ("need_off", "seq_off", "kind", "start", "end", "sr_off", "sr_n", "s_start", "s_end"):
        assert np.array_equal(got[k].cpu().numpy().astype(np.uint64), exp[k].astype(np.uint64)), k


@pytest.mark.parametrize("case", SYNC["cases"], ids=[c["name"] for c in SYNC["cases"]])
def test_sync_kats_gpu_1pass(case):
    from corrosion_amd.sync import _needs_device_1pass
    ent = entries_from_pairs([(case["our"], case["their"])])
    got = {k: v.cpu().numpy().astype(np.uint64) for k, v in _needs_device_1pass(_engine(), _to_dev(ent)).items()}
    assert decode_needs(got, 1)[0] == kat_expect(case["expect"])


def test_sync_random_vs_oracle_1pass():
    rng = np.random.default_rng(6)
    pairs = [(random_side(rng, with_head=rng.random() < 0.9), random_side(rng)) for _ in range(40000)]
    _check_1pass(entries_from_pairs(pairs))   # 157 workgroups: look-back spans several waves


def test_sync_config4_shape_1pass_equals_two_pass():
    """Config-4-shaped entries in HBM (600K entries, 2344 workgroups): the one-pass kernel's CSR
    equals the two-pass kernel's and the oracle's."""
    import synth
    from corrosion_amd.sync import _needs_device, _needs_device_1pass
    ent = synth.sync_entries_torch(20000, 30, 21, device="cuda")
    e = _engine()
    a = _needs_device(e, ent)
    b = _needs_device_1pass(e, ent)
    for k in a:
        assert a[k].shape == b[k].shape and bool((a[k] == b[k]).all()), k
    exp = O.needs({k: v.cpu().numpy() for k, v in ent.items()})
    for k in ("need_off", "kind", "start", "s_end"):
        assert np.array_equal(b[k].cpu().numpy().astype(np.uint64), exp[k].astype(np.uint64)), k


@pytest.mark.parametrize("dense", ["theirs", "ours", "both"])
def test_sync_lds_caps_exceeded_1pass(dense):
    rng = np.random.default_rng(12)
    pairs = []
    for i in range(1200):
        heavy = 256 <= i < 768
        nt = 12 if heavy and dense in ("theirs", "both") else int(rng.poisson(2))
        no = 12 if heavy and dense in ("ours", "both") else int(rng.poisson(2))
        pairs.append((_dense_side(rng, no, int(rng.integers(1, 100))), _dense_side(rng, nt, 300)))
    _check_1pass(entries_from_pairs(pairs))


def test_sync_1pass_capacity_error_reports_totals():
    """Caps below the output size: CORRO_E_RANGE, the exact totals, no write past the caps; the
    wrapper's re-run at those totals gives the oracle's result (here with overlapping our-need
    ranges, which the RangeInclusiveSet-based bound does not cover)."""
    import ctypes as C
    import torch
    import corrosion_amd._lib as L
    their = {"head": 400, "need": [[k, k] for k in range(3, 390, 4)], "partials": {}}
    our = {"head": None, "need": [[1, 395]] * 6, "partials": {}}
    ent = entries_from_pairs([(our, their)] * 300)
    _check_1pass(ent)
    d = _to_dev(ent)
    e = _engine()
    s = L.SyncEntries()
    s.n = len(ent["their_head"])
    for k, _ in L.SyncEntries._fields_[1:]:
        setattr(s, k, d[k].data_ptr() if d[k].numel() else None)
    o = L.NeedsOut()
    guard = torch.full((64,), 7, dtype=torch.int64, device="cuda")
    bufs = {k: torch.zeros(s.n + 1, dtype=torch.int64, device="cuda") for k in ("need_off", "seq_off")}
    for k in ("need_off", "seq_off"):
        setattr(o, k, bufs[k].data_ptr())
    for k in ("kind", "start", "end", "sr_off", "sr_n", "s_start", "s_end"):
        setattr(o, k, guard.data_ptr())
    tot = (C.c_uint64 * 2)()
    rc = L.lib().corro_compute_needs_onepass(e._h, C.byref(s), C.byref(o), 0, 0, tot)
    assert rc == -6
    exp = O.needs(ent)
    assert tot[0] == int(exp["need_off"][-1]) and tot[1] == int(exp["seq_off"][-1])
    assert bool((guard == 7).all())


def test_inverted_our_need_ranges_vs_fixture():
    """The three config-4 entries (found at full size) whose our-need list holds an inverted range."""
    from tests.sync_util import expected_from_cases, pairs_from_cases
    cases = load_golden("sync_inverted_cases.json")["cases"]
    e = _engine()
    got = decode_needs(e.compute_needs(entries_from_pairs(pairs_from_cases(cases))), len(cases))
    assert got == expected_from_cases(cases)


# ---- packed one-pass form (corro_compute_needs_packed: bound-reserved slots, no count pass) -----

def _packed_csr(ent_dev):
    from corrosion_amd.sync import _needs_device_packed, packed_to_csr
    return packed_to_csr(_needs_device_packed(_engine(), ent_dev))


def _check_packed(ent_host):
    got = _packed_csr(_to_dev(ent_host))
    exp = O.needs(ent_host)
    for k in ("need_off", "seq_off", "kind", "start", "end", "sr_off", "sr_n", "s_start", "s_end"):
        assert np.array_equal(got[k].astype(np.uint64), exp[k].astype(np.uint64)), k


@pytest.mark.parametrize("case", SYNC["cases"], ids=[c["name"] for c in SYNC["cases"]])
def test_sync_kats_gpu_packed(case):
    ent = entries_from_pairs([(case["our"], case["their"])])
    assert decode_needs(_packed_csr(_to_dev(ent)), 1)[0] == kat_expect(case["expect"])


def test_sync_random_vs_oracle_packed():
    rng = np.random.default_rng(16)
    pairs = [(random_side(rng, with_head=rng.random() < 0.9), random_side(rng)) for _ in range(40000)]
    _check_packed(entries_from_pairs(pairs))


@pytest.mark.parametrize("dense", ["theirs", "ours", "both"])
def test_sync_lds_caps_exceeded_packed(dense):
    """Workgroups whose segments exceed the LDS caps walk global memory; same result."""
    rng = np.random.default_rng(13)
    pairs = []
    for i in range(1200):
        heavy = 256 <= i < 768
        nt = 12 if heavy and dense in ("theirs", "both") else int(rng.poisson(2))
        no = 12 if heavy and dense in ("ours", "both") else int(rng.poisson(2))
        pairs.append((_dense_side(rng, no, int(rng.integers(1, 100))), _dense_side(rng, nt, 300)))
    _check_packed(entries_from_pairs(pairs))


def test_sync_config4_shape_packed_vs_oracle():
    import synth
    ent = synth.sync_entries_torch(20000, 30, 22, device="cuda")
    got = _packed_csr(ent)
    exp = O.needs({k: v.cpu().numpy() for k, v in ent.items()})
    for k in ("need_off", "seq_off", "kind", "start", "end", "sr_off", "sr_n", "s_start", "s_end"):
        assert np.array_equal(got[k].astype(np.uint64), exp[k].astype(np.uint64)), k


def test_sync_packed_overlapping_ranges_rejected():
    """Overlapping our-need ranges (no RangeInclusiveSet produces them) can exceed the bound slots:
    CORRO_E_RANGE instead of a write past a workgroup's slots."""
    from corrosion_amd.sync import _needs_device_packed
    their = {"head": 400, "need": [[k, k] for k in range(3, 390, 4)], "partials": {}}
    our = {"head": None, "need": [[1, 395]] * 6, "partials": {}}
    ent = entries_from_pairs([(our, their)] * 300)
    with pytest.raises(RuntimeError, match="CORRO_E_RANGE"):
        _needs_device_packed(_engine(), _to_dev(ent))
