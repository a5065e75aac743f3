"""CPU check (oracle against itself) of the overflow fold's row reduction (ovf_kernels.h, k_ovf_lookup's
comment): without impacts, a row whose records all satisfy SURVEY App. A.3, whose largest cl Mx is
even, or whose cids all have a change with col_version > 0 at Mx, folds to the same crsql_changes rows
from its changes at cl == Mx alone. The sequential fold (oracle/crsql_fold.c, cr-sqlite's rules of
/root/reference/crates/corro-agent/src/agent/util.rs:1225-1245) is run on the whole batch and on the
reduced one, into the same prior state, and the rows must be identical."""
import numpy as np
import pytest

import synth
from oracle import oracle as O
from tests._util import rows_to_tuples


def reduce_keep(batch, prior):
    """The engine's keep mask over `batch` (k_ovf_rfin / k_ovf_keep restated with numpy), the
    prior state's clock rows counted in each row's summary like the prior records the fold appends."""
    def cols(b, is_prior):
        cid = (b["table_cid"] & 0xFFFF).astype(np.int64)
        cl = b["cl"].astype(np.int64)
        cv = b["col_version"].astype(np.int64)
        bad = ((cid == 0) | ((cl & 1) == 0)) & (cv != cl)
        if is_prior:
            bad |= (cid != 0) & ((cl & 1) == 0)
        return b["table_cid"] >> 16, b["pk"].astype(np.uint64), cid, cl, cv, bad

    parts = [cols(batch, False)] + ([cols(prior, True)] if prior is not None and len(prior["pk"]) else [])
    t, pk, cid, cl, cv, bad = (np.concatenate([p[i] for p in parts]) for i in range(6))
    rows, inv = np.unique(np.stack([t.astype(np.uint64), pk]), axis=1, return_inverse=True)
    inv = inv.reshape(-1)
    nr = rows.shape[1]
    mx = np.zeros(nr, np.int64)
    np.maximum.at(mx, inv, cl)
    rbad = np.zeros(nr, bool)
    np.logical_or.at(rbad, inv, bad)
    bit = np.where(cid != 0, np.left_shift(np.uint64(1), cid.astype(np.uint64) & np.uint64(63)), np.uint64(0))
    call = np.zeros(nr, np.uint64)
    np.bitwise_or.at(call, inv, bit)
    fin = (cid != 0) & (cv > 0) & (cl == mx[inv])
    cfin = np.zeros(nr, np.uint64)
    np.bitwise_or.at(cfin, inv, np.where(fin, bit, np.uint64(0)))
    red = ~rbad & (((mx & 1) == 0) | (cfin == call))
    keep = ~red[inv] | (cl == mx[inv])
    return keep[: len(batch["pk"])], red


def _sub(b, m):
    return {k: (v[m] if isinstance(v, np.ndarray) and v.shape[:1] == m.shape else v) for k, v in b.items()}


@pytest.mark.parametrize("seed,npk,malformed", [(1, 64, False), (2, 512, False), (3, 64, True), (4, 4096, False)])
def test_row_reduction_equals_full_fold(seed, npk, malformed):
    sites = synth.site_ids(16, seed)
    b1 = synth.adversarial_batch(20000, 16, 3, npk, seed, malformed=malformed)
    b2 = synth.adversarial_batch(40000, 16, 3, npk, seed + 100, malformed=malformed)
    full, red = O.Fold(sites), O.Fold(sites)
    for f in (full, red):
        f.apply(b1)
    prior = full.export()
    keep, rows_reduced = reduce_keep(b2, prior)
    full.apply(b2)
    red.apply(_sub(b2, keep))
    if not malformed:  # the rule fires on hot rows (malformed ones keep every change)
        assert rows_reduced.sum() > 0 and (~keep).sum() > len(keep) // 4
    assert rows_to_tuples(red.export(), with_ts=True) == rows_to_tuples(full.export(), with_ts=True)


def test_row_reduction_empty_prior():
    sites = synth.site_ids(8, 7)
    b = synth.adversarial_batch(30000, 8, 2, 32, 7)
    keep, _ = reduce_keep(b, None)
    full, red = O.Fold(sites), O.Fold(sites)
    full.apply(b)
    red.apply(_sub(b, keep))
    assert (~keep).sum() > len(keep) // 2
    assert rows_to_tuples(red.export(), with_ts=True) == rows_to_tuples(full.export(), with_ts=True)


@pytest.mark.parametrize("max_cl,sentinel_frac", [(12, 0.3), (3, 0.6), (20, 0.1)])
def test_row_reduction_epoch_mixes(max_cl, sentinel_frac):
    """Many epochs per row (up to 20 causal lengths), delete-heavy and resurrect-heavy mixes, three
    batches folded: the reduced batch always gives the full batch's rows."""
    seed = 40 + max_cl
    sites = synth.site_ids(12, seed)
    full, red = O.Fold(sites), O.Fold(sites)
    for k in range(3):
        b = synth.adversarial_batch(25000, 12, 2, 128, seed * 7 + k, max_cl=max_cl, sentinel_frac=sentinel_frac)
        keep, _ = reduce_keep(b, full.export())
        full.apply(b)
        red.apply(_sub(b, keep))
        assert rows_to_tuples(red.export(), with_ts=True) == rows_to_tuples(full.export(), with_ts=True), k
