"""oracle.rows_diff: the row-by-row report a failed full-size parity check prints (CPU)."""
import numpy as np

import synth
from oracle import oracle as O


def _state(seed, shards=False):
    sites = synth.site_ids(16, 3)
    b = synth.uniform_batch(20_000, 16, 500, 4, seed)
    f = O.ShardedFold(sites, nshards=4, nthreads=2) if shards else O.Fold(sites)
    f.apply(b)
    return f


def test_equal_states_report_nothing():
    a, b = _state(5).export(), _state(5, shards=True).export()
    assert O.rows_diff(a, b) is None
    assert O.rows_digest(a) == _state(5, shards=True).digest()


def test_changed_field_and_missing_row_are_named():
    ref = _state(6).export()
    got = {k: (v.copy() if isinstance(v, np.ndarray) else dict(v)) for k, v in ref.items()}
    got["col_version"][7] += 1
    rep = O.rows_diff(got, ref)
    assert rep and "1 of" in rep and "col_version" in rep and f"pk {int(ref['pk'][7])}" in rep
    cut = {k: (np.delete(v, 3) if isinstance(v, np.ndarray) else {}) for k, v in ref.items()}
    rep = O.rows_diff(cut, ref)
    assert rep and "missing row" in rep and f"pk {int(ref['pk'][3])}" in rep
