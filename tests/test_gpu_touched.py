"""Per-apply delta export (corro_state_export_touched) and failure atomicity.

A drop-in must keep SQLite as the durable state: every reference INSERT INTO crsql_changes writes the
clock (and base) rows inside the caller's transaction (/root/reference/crates/corro-agent/src/agent/
util.rs:749-758, :1225-1245). The engine returns, after each apply, the complete clock set of every
row it addressed; a host table kept by replacing those rows must equal the whole-state export after
any sequence of applies (deletes / resurrects included, so the replacement semantics matter).
"""
import numpy as np
import pytest

import corrosion_amd as ca
import synth
from tests._util import rows_to_tuples

pytestmark = pytest.mark.gpu


def _canon(rows):
    """{(table, pk): sorted row tuples} with long values by their bytes"""
    longs = rows.get("long_values", {})
    keys = ("table_cid", "pk", "val_type", "val0", "val1", "val_len", "col_version", "db_version", "site", "cl",
            "seq", "ts")
    cols = [np.asarray(rows[k]).tolist() for k in keys]
    for i, b in longs.items():
        cols[4][i] = b
    out = {}
    for t in zip(*cols):
        out.setdefault((t[0] >> 16, t[1]), []).append(t)
    return {k: sorted(v, key=repr) for k, v in out.items()}


def _replay(host, delta):
    """a host store kept by DELETE WHERE key = pk; INSERT the row's exported clocks"""
    for key, rows in _canon(delta).items():
        host[key] = rows


@pytest.mark.parametrize("long_values", [False, True])
def test_deltas_rebuild_the_state(long_values):
    sites = synth.site_ids(16, 5)
    schema = synth.adversarial_schema(8)
    eng = ca.MergeEngine(schema, capacity_hint=1 << 16)
    eng.register_sites(sites)
    eng.track_touched(True)
    host = {}
    for k in range(5):
        b = synth.adversarial_batch(60000, 16, 8, 3000, 40 + k)
        if long_values:
            b = synth.with_long_values(b, 50 + k)
        eng.apply(b, impact=(k % 2 == 0))
        d = eng.export_touched()
        assert len(d["pk"]) <= eng.count()
        _replay(host, d)
        assert len(eng.export_touched()["pk"]) == 0          # consumed
    assert host == _canon(eng.export())


def test_delta_scales_with_touched_rows():
    """a small batch into a large state exports only its rows"""
    sites = synth.site_ids(8, 6)
    eng = ca.MergeEngine({"t": ["a", "b", "c", "d"]}, capacity_hint=1 << 20)
    eng.register_sites(sites)
    eng.track_touched(True)
    eng.apply(synth.uniform_batch(1 << 20, 8, 1 << 18, 4, 7))
    big = eng.export_touched()
    small = synth.uniform_batch(1000, 8, 1 << 18, 4, 8)
    eng.apply(small)
    d = eng.export_touched()
    rows = {(int(t) >> 16, int(p)) for t, p in zip(d["table_cid"], d["pk"])}
    assert rows == {(0, int(p)) for p in small["pk"]}
    assert len(d["pk"]) <= 5 * len(rows) < len(big["pk"]) // 100
    full = _canon(eng.export())
    for key, rr in _canon(d).items():
        assert full[key] == rr


def test_delta_through_process_multiple_changes():
    """the agent path: the delta of one call holds the rows its complete versions merged"""
    from corrosion_amd.agent import Agent, Change, ChangeV1, Full
    a = Agent({"t": ["x", "y"]}, capacity_hint=1 << 12)
    a.engine.track_touched(True)
    A = bytes([7] * 16)
    cs = [ChangeV1(A, Full(v, [Change("t", v % 3, "x", v, 1, v, 0, A, 1)], (0, 0), 0, ts=v)) for v in range(1, 6)]
    a.process_multiple_changes(cs)
    d = a.engine.export_touched()
    assert sorted({int(p) for p in d["pk"]}) == [0, 1, 2]
    assert _canon(d) == _canon(a.engine.export())


def test_mid_apply_failure_poisons_until_reset():
    """a resource limit hit after the merge began writing cannot be rolled back in place;
    the context refuses every later call until corro_state_reset, then works again."""
    sites = synth.site_ids(4, 7)
    eng = ca.MergeEngine({"t": ["a", "b", "c", "d"]}, capacity_hint=1 << 12)
    eng.register_sites(sites)
    eng.set_store_limit(1)                    # no heap growth at all
    b = synth.uniform_batch(200000, 4, 150000, 4, 9)
    with pytest.raises(ca.CorroError, match="poisoned"):
        eng.apply(b)
    with pytest.raises(ca.CorroError, match="poisoned"):
        eng.apply(synth.uniform_batch(10, 4, 100, 4, 10))
    with pytest.raises(ca.CorroError, match="poisoned"):
        eng.export()
    eng.reset()
    eng.set_store_limit(0)
    small = synth.uniform_batch(1000, 4, 100, 4, 11)
    eng.apply(small)
    from oracle import oracle as O
    f = O.Fold(sites)
    f.apply(small)
    assert sorted(rows_to_tuples(eng.export())) == sorted(rows_to_tuples(f.export()))


def test_failure_before_writes_does_not_poison():
    eng = ca.MergeEngine({"t": ["a"]}, capacity_hint=1 << 12)
    eng.register_sites(synth.site_ids(2, 8))
    ok = synth.uniform_batch(100, 2, 50, 1, 12)
    eng.apply(ok)
    bad = synth.uniform_batch(100, 2, 50, 1, 13)
    bad["table_cid"][5] = 7                     # unknown column: refused before any write
    with pytest.raises(ca.CorroError, match="UNKNOWN_COLUMN"):
        eng.apply(bad)
    eng.apply(synth.uniform_batch(100, 2, 50, 1, 14))     # still usable


def test_affinity_check_with_out_of_range_long_value():
    """a long TEXT value whose val_off points past val_data on a table with registered
    affinities is reported as malformed (CORRO_E_INVALID), never read out of bounds."""
    from tests.test_gpu_affinity import _batch, _engine
    e, _f = _engine()
    b = _batch([(1, 1, "abc")])
    b["val_len"][0] = 255
    b["val_off"] = np.array([1 << 40], np.uint64)
    b["val_size"] = np.array([40], np.uint32)
    b["val_data"] = np.frombuffer(b"x" * 40, np.uint8).copy()
    with pytest.raises(ca.CorroError, match="CORRO_E_INVALID"):
        e.apply(b)
    e.apply(_batch([(2, 3, "fine")]))
