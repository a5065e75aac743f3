"""TEXT / BLOB values of any length (SqliteValue::Text(String) / Blob(Vec<u8>),
/root/reference/crates/corro-api-types/src/lib.rs:419-429) through every merge path: values longer
than 16 bytes live in the device value arena and compare by their whole bytes (memcmp, then length),
as cr-sqlite's merge-equal-values tie-break does. Checked bit-exact against the oracle (whose
arena holds the same bytes), with impacts, across batches (long values already in the state),
chunked applies, device-resident batches, the overflow path, and the agent + handle_need path."""
import numpy as np
import pytest

import synth
from oracle import oracle as O
from tests._util import rows_to_tuples

pytestmark = pytest.mark.gpu

SCHEMA = {"t": ["a", "b", "c", "d"]}


def _engine(schema, sites, cap=1 << 16):
    import corrosion_amd as ca
    e = ca.MergeEngine(schema, capacity_hint=cap)
    e.register_sites(sites)
    return e


def _compare(e, f, with_ts=False):
    got, exp = e.export(), f.export()
    assert rows_to_tuples(got, with_ts) == rows_to_tuples(exp, with_ts)
    assert O.rows_digest(got) == O.rows_digest(exp)
    assert list(e.db_versions()[:f.nsites]) == list(f.db_versions())
    return got


@pytest.mark.parametrize("impact", [False, True])
def test_long_values_cl1_batches_vs_oracle(impact):
    """cl = 1 changes (fast-path shape) with long values: their buckets take the general body, and a
    region that holds a long value keeps later batches off the fast bodies."""
    sites = synth.site_ids(8, 5)
    e, f = _engine(SCHEMA, sites), O.Fold(sites)
    for k in range(4):
        b = synth.uniform_batch(20000, 8, 3000, 4, 60 + k, cv_max=2, tie_frac=0.5)
        b = synth.with_long_values(b, 70 + k, frac=0.1 if k < 3 else 0.0)
        ie = e.apply(b, impact=impact)
        jf = f.apply(b)
        if impact:
            assert np.array_equal(ie, jf)
        got = _compare(e, f)
    assert len(got["long_values"]) > 100


@pytest.mark.parametrize("seed", [81, 82])
def test_long_values_adversarial_vs_oracle(seed):
    """Deletes / resurrects / sentinels with long values (general body)."""
    sites = synth.site_ids(8, seed)
    e, f = _engine(synth.adversarial_schema(2), sites, cap=30000), O.Fold(sites)
    for k in range(2):
        b = synth.with_long_values(synth.adversarial_batch(30000, 8, 2, 500, seed + 10 * k), seed + k, frac=0.3)
        assert np.array_equal(e.apply(b, impact=True), f.apply(b))
        _compare(e, f, with_ts=True)


def test_long_values_overflow_path_vs_oracle():
    """Zipf-hot rows in a tiny bucket table: the device-wide overflow fold compares long values."""
    seed = 91
    sites = synth.site_ids(8, seed)
    b = synth.with_long_values(synth.adversarial_batch(60000, 8, 1, 60, seed, zipf=1.1), seed, frac=0.4)
    e, f = _engine(synth.adversarial_schema(1), sites, cap=64), O.Fold(sites)
    assert np.array_equal(e.apply(b, impact=True), f.apply(b))
    _compare(e, f, with_ts=True)
    b2 = synth.with_long_values(synth.adversarial_batch(60000, 8, 1, 60, seed + 1, zipf=1.1), seed + 1, frac=0.4)
    assert np.array_equal(e.apply(b2, impact=True), f.apply(b2))
    _compare(e, f, with_ts=True)


def test_long_values_chunked_apply(monkeypatch):
    monkeypatch.setenv("CORRO_HIP_CHUNK", "4096")
    sites = synth.site_ids(8, 7)
    b = synth.with_long_values(synth.adversarial_batch(40000, 8, 1, 2000, 7, zipf=0.5), 8, frac=0.3)
    e, f = _engine(synth.adversarial_schema(1), sites, cap=40000), O.Fold(sites)
    assert np.array_equal(e.apply(b, impact=True), f.apply(b))
    _compare(e, f, with_ts=True)


def test_long_values_device_batch():
    import torch
    sites = synth.site_ids(8, 9)
    b = synth.with_long_values(synth.uniform_batch(50000, 8, 5000, 4, 9, cv_max=2), 10, frac=0.2)

    def dev(v):
        v = np.ascontiguousarray(v)
        if v.dtype == np.uint64:
            v = v.view(np.int64)
        elif v.dtype == np.uint32:
            v = v.view(np.int32)
        return torch.from_numpy(v.copy()).cuda()
    d = {k: dev(v) for k, v in b.items()}
    e, f = _engine(SCHEMA, sites, cap=50000), O.Fold(sites)
    ie = e.apply(d, impact=True)
    assert np.array_equal(ie.cpu().numpy(), f.apply(b))
    _compare(e, f)


def test_malformed_long_values_are_rejected_and_leave_state_untouched():
    import corrosion_amd as ca
    sites = synth.site_ids(4, 3)
    e = _engine(SCHEMA, sites)
    good = synth.with_long_values(synth.uniform_batch(1000, 4, 100, 4, 3), 4, frac=0.3)
    e.apply(good)
    before = rows_to_tuples(e.export())
    for bad_k in ("short", "span", "nodata"):
        b = synth.with_long_values(synth.uniform_batch(1000, 4, 100, 4, 5), 6, frac=0.3)
        i = int(np.nonzero(b["val_len"] == 255)[0][3])
        b["val_size"] = b["val_size"].copy()
        b["val_off"] = b["val_off"].copy()
        if bad_k == "short":
            b["val_size"][i] = 16          # a long value must be longer than 16 bytes
        elif bad_k == "span":
            b["val_off"][i] = len(b["val_data"])  # bytes past val_data
        else:
            b = {k: v for k, v in b.items() if k not in ("val_off", "val_size", "val_data")}
        with pytest.raises(ca.CorroError):
            e.apply(b)
        assert rows_to_tuples(e.export()) == before


def test_agent_long_values_round_trip_through_handle_need():
    """process_multiple_changes with long TEXT / BLOB values, then handle_need serves them back
    whole (crsql_changes rows -> Change objects with the full bytes)."""
    from corrosion_amd.agent import Agent, Change, ChangeV1, Full
    from corrosion_amd.sync import Full as NeedFull
    a = Agent({"tests": ["text", "blob"]}, capacity_hint=1 << 12)
    actor = bytes([7]) * 16
    long_t = "a text value that is much longer than sixteen bytes " * 3
    long_b = bytes(range(256)) * 2
    ch = [Change("tests", 1, "text", long_t, 1, 1, 0, actor, 1),
          Change("tests", 1, "blob", long_b, 1, 1, 1, actor, 1),
          Change("tests", 2, "text", "short", 1, 1, 2, actor, 1)]
    r = a.process_multiple_changes([ChangeV1(actor, Full(version=1, changes=ch, seqs=(0, 2), last_seq=2, ts=5))])
    assert r.known == ["current"]
    # a later version: a longer value with the same 52-byte prefix wins at equal col_version
    ch2 = [Change("tests", 1, "text", long_t + "!", 1, 2, 0, actor, 1)]
    r = a.process_multiple_changes([ChangeV1(actor, Full(version=2, changes=ch2, seqs=(0, 0), last_seq=0, ts=6))])
    assert r.impactful == [ch2]
    out = a.handle_needs([(actor, NeedFull(1, 2))])[0]
    vals = {(c.pk, c.cid): c.val for m in out for c in m.changeset.changes}
    assert vals[(1, "text")] == long_t + "!"
    assert vals[(1, "blob")] == long_b
    assert vals[(2, "text")] == "short"
