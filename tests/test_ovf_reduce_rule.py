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


# ---- impacts of a reduced row's dropped changes (the overflow fold's impact form) ---------------
NCL = 8       # causal-length slots per row (ovf_kernels.h OVF_NCL): more distinct cls keep every record
PM = 1 << 20  # compact position of batch change i: PM + i (prior clock records: their cid slot)


def _vkey(t, v0, v1, vl, cv, site_id):
    """a change's cell key as cr-sqlite orders it: (col_version, value by type rank then payload,
    writer site id) -- oracle/crsql_fold.c value_cmp"""
    t = int(t)
    if t == 1:
        p = int(np.int64(np.uint64(v0)))
    elif t == 2:
        p = float(np.uint64(v0).view(np.float64))
    elif t in (3, 4):
        p = (int(v0).to_bytes(8, "big") + int(v1).to_bytes(8, "big"))[:int(vl)]
    else:
        p = 0
    return (int(cv), 5 - t, p, bytes(site_id))


def reduce_impacts(batch, prior, site_ids):
    """The overflow fold's impact flags with the row reduction (ovf_kernels.h, k_ovf_keep's impact
    form) restated: returns (keep mask over the batch, impact flags of the DROPPED changes, NaN
    elsewhere). Per reduced row, with F(c) the first compact position of causal length c and H(c) the
    first position of any larger one, a dropped change at position p with causal length c is
      a record  (p == F(c) < H(c)): 1, or 2 for a column change with odd c > 1 (a resurrect);
      a candidate (F(c) < p < H(c), odd c, column change): 1 iff its key beats every earlier
        candidate of its (row, c, cid) group and the epoch record's own key when that record is a
        column change of the same cid (a carried, zeroed cell loses to any col_version > 0);
      a no-op otherwise: 0."""
    recs = []  # (row key, pos, cid, cl, cv, key, batch index or -1)
    if prior is not None:
        for k in range(len(prior["pk"])):
            cid = int(prior["table_cid"][k]) & 0xFFFF
            recs.append(((int(prior["table_cid"][k]) >> 16, int(prior["pk"][k])), cid, cid,
                         int(prior["cl"][k]), int(prior["col_version"][k]),
                         _vkey(prior["val_type"][k], prior["val0"][k], prior["val1"][k], prior["val_len"][k],
                               prior["col_version"][k], site_ids[int(prior["site"][k])]), -1))
    n = len(batch["pk"])
    for i in range(n):
        cid = int(batch["table_cid"][i]) & 0xFFFF
        recs.append(((int(batch["table_cid"][i]) >> 16, int(batch["pk"][i])), PM + i, cid, int(batch["cl"][i]),
                     int(batch["col_version"][i]),
                     _vkey(batch["val_type"][i], batch["val0"][i], batch["val1"][i], batch["val_len"][i],
                           batch["col_version"][i], site_ids[int(batch["site"][i])]), i))
    rows = {}
    for r in recs:
        rows.setdefault(r[0], []).append(r)
    keep = np.ones(n, bool)
    imp = np.full(n, np.nan)
    for rk, rr in rows.items():
        rr.sort(key=lambda r: r[1])
        mx = max(r[3] for r in rr)
        bad = any(((r[2] == 0 or r[3] % 2 == 0) and r[4] != r[3]) or (r[6] < 0 and r[2] != 0 and r[3] % 2 == 0)
                  or (r[6] >= 0 and r[2] != 0 and r[4] <= 0) for r in rr)
        cls = sorted({r[3] for r in rr})
        bad |= len(cls) > NCL
        call = {r[2] for r in rr if r[2] != 0}
        fin = {r[2] for r in rr if r[2] != 0 and r[4] > 0 and r[3] == mx}
        if bad or not (mx % 2 == 0 or fin == call):
            continue
        F = {}
        for r in rr:
            F.setdefault(r[3], r)       # first record of each causal length (rr is in position order)
        best = {}                        # (c, cid) -> running max key of the group
        for r in rr:
            c, cid, p, i = r[3], r[2], r[1], r[6]
            if c == mx:
                continue
            if i >= 0:
                keep[i] = False
            H = min((F[x][1] for x in cls if x > c), default=1 << 62)
            f = F[c]
            if p == f[1] and p < H:
                out = 2 if (cid != 0 and c % 2 and c > 1) else 1
            elif f[1] < p < H and c % 2 and cid != 0:
                g = (c, cid)
                if g not in best:
                    best[g] = f[5] if (f[2] == cid) else None
                out = 1 if best[g] is None or r[5] > best[g] else 0
                if best[g] is None or r[5] > best[g]:
                    best[g] = r[5]
            else:
                out = 0
            if i >= 0:
                imp[i] = out
    return keep, imp


@pytest.mark.parametrize("seed,npk,max_cl,sent", [(1, 64, 6, 0.3), (2, 512, 6, 0.3), (3, 48, 7, 0.3),
                                                  (4, 96, 3, 0.6), (5, 32, 20, 0.1), (6, 40, 12, 0.3)])
def test_row_reduction_impacts_equal_full_fold(seed, npk, max_cl, sent):
    """With impacts: the full batch's crsql_rows_impacted() flags equal the reduced batch's flags on
    the kept changes and reduce_impacts' flags on the dropped ones, and the rows are equal; two batches
    (the second onto the first's state, whose clock rows enter each row's summary as prior records)."""
    sites = synth.site_ids(16, seed)
    full, red = O.Fold(sites), O.Fold(sites)
    for k in range(2):
        b = synth.adversarial_batch(20000, 16, 3, npk, seed * 10 + k, wide=False, max_cl=max_cl, sentinel_frac=sent)
        keep, dimp = reduce_impacts(b, full.export() if k else None, sites)
        want = full.apply(b)
        got = np.zeros(len(keep), np.int64)
        got[keep] = red.apply(_sub(b, keep))
        got[~keep] = dimp[~keep]
        if max_cl <= NCL:  # (rows with more distinct causal lengths than slots keep every change)
            assert (~keep).sum() > len(keep) // 4
        assert np.array_equal(got, want), (k, np.flatnonzero(got != want)[:10])
        assert rows_to_tuples(red.export(), with_ts=True) == rows_to_tuples(full.export(), with_ts=True), k
