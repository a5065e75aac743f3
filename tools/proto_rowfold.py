"""Prototype (CPU, test tooling) of the parallel per-row fold that the general merge body uses for
long rows, checked against the sequential oracle (oracle/crsql_fold.c) on random batches.

Per row, with changes in application order (prior state first, as a prefix):
  L_i      = exclusive running max of cl                      (a segmented max-scan)
  record   = cl_i > L_i;  dead = cl_i < L_i;  candidate = cl_i == L_i, odd, column change
  epochs   = the records, in order (L only grows: few per row)
  W(e, c)  = argmax of the epoch's candidates of cid c by (cv, value, site), earliest on ties
             (a reduction: order-free)
  then one sequential walk over the row's records only (not its changes): delete records drop
  the cells, odd records zero them (carried, cv -> 0) and a column record sets its own cell, and
  each epoch's W(e, c) replaces the carried cell when strictly greater.
  impact: records 1 (2 for a column record that resurrects), candidates 1 iff strictly greater
  than the epoch's first element of that cell (the record's cell or the zeroed carried one) and
  every earlier candidate of that cell (a segmented prefix max), else 0.
Valid when every sentinel / even-cl change carries col_version == cl; other rows
keep the sequential fold.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def vkey(t, v0, v1, ln):
    rank = 5 - t
    if t == 1:
        k0 = (int(v0) ^ (1 << 63))
    elif t == 2:
        x = int(v0)
        if x == 1 << 63:
            x = 0
        k0 = ((~x) & ((1 << 64) - 1)) if (x >> 63) else (x | (1 << 63))
    elif t in (3, 4):
        k0 = int(v0)
    else:
        k0 = 0
    if t in (3, 4):
        return (rank, k0, int(v1), int(ln))
    return (rank, k0, 0, 0)


def key(c, zeroed=False):
    return (0 if zeroed else c["cv"], vkey(c["t"], c["v0"], c["v1"], c["ln"]), c["site"])


def fold_row(chs):
    """chs: list of dicts (application order). Returns (rows, impacts) or None (fallback)."""
    for c in chs:
        if (c["cid"] == 0 or c["cl"] % 2 == 0) and c["cv"] != c["cl"]:
            return None
    L, Ls = 0, []
    for c in chs:
        Ls.append(L)
        L = max(L, c["cl"])
    Lf = L
    n = len(chs)
    kind = []
    for i, c in enumerate(chs):
        if c["cl"] > Ls[i]:
            kind.append("rec")
        elif c["cl"] < Ls[i]:
            kind.append("dead")
        elif c["cid"] != 0 and c["cl"] % 2 == 1:
            kind.append("cand")
        else:
            kind.append("noop")
    recs = [i for i in range(n) if kind[i] == "rec"]
    # epoch index per change: index of the last record at or before it
    ep, e = [], -1
    for i in range(n):
        if kind[i] == "rec":
            e += 1
        ep.append(e)
    # W(e, c): order-free argmax, earliest on ties
    W = {}
    for i in range(n):
        if kind[i] != "cand":
            continue
        g = (ep[i], chs[i]["cid"])
        if g not in W or key(chs[i]) > key(chs[W[g]]):
            W[g] = i
    # sequential walk over records
    state = {}  # cid -> (idx, zeroed)
    first = {}  # (e, cid) -> key of the epoch's first element for that cell
    imp = [0] * n
    for e, r in enumerate(recs):
        R = chs[r]
        if R["cl"] % 2 == 0:
            state = {}
            imp[r] = 1
        else:
            state = {c: (j, True) for c, (j, _) in state.items()}
            if R["cid"] != 0:
                imp[r] = (1 if (Ls[r] > 0 or R["cl"] > 1) else 0) + 1
                state[R["cid"]] = (r, False)
            else:
                imp[r] = 1
            for c, (j, z) in state.items():
                first[(e, c)] = key(chs[j], z)
            for (ee, c), w in W.items():
                if ee != e:
                    continue
                cur = state.get(c)
                if cur is None or key(chs[w]) > key(chs[cur[0]], cur[1]):
                    state[c] = (w, False)
    # candidate impacts: strict prefix max within (epoch, cid), seeded by the epoch's first element
    best = {}
    for i in range(n):
        if kind[i] != "cand":
            continue
        g = (ep[i], chs[i]["cid"])
        k = key(chs[i])
        m = best.get(g, first.get(g))
        if m is None or k > m:
            imp[i] = 1
            best[g] = k
    rows = []
    r = recs[-1]
    R = chs[r]
    has_sent = not (R["cid"] != 0 and R["cl"] == 1 and Ls[r] == 0)
    if has_sent:
        rows.append(dict(R, cid=0, cv=R["cv"] if R["cid"] == 0 else R["cl"], t=5, v0=0, v1=0, ln=0))
    rowcl = rows[0]["cv"] if has_sent else 1
    if Lf % 2 == 1:
        for c, (j, z) in state.items():
            rows.append(dict(chs[j], cid=c, cv=0 if z else chs[j]["cv"]))
    for x in rows:
        x["rowcl"] = rowcl
    return rows, imp


def check(batch, sites, prior=None):
    from oracle import oracle as O
    n = len(batch["pk"])
    f = O.Fold(sites)
    if prior is not None:
        f.apply(prior)
        pre = f.export()
    imp_ref = f.apply(batch)
    ref = f.export()
    # group by row, prior state first (as a prefix: sentinel first)
    rows = {}
    if prior is not None:
        m = len(pre["pk"])
        order = sorted(range(m), key=lambda k: (int(pre["table_cid"][k]) >> 16, int(pre["pk"][k]),
                                                 0 if (int(pre["table_cid"][k]) & 0xFFFF) == 0 else 1))
        for k in order:
            tc = int(pre["table_cid"][k])
            c = dict(pk=int(pre["pk"][k]), table=tc >> 16, cid=tc & 0xFFFF, cl=int(pre["cl"][k]),
                     cv=int(pre["col_version"][k]), t=int(pre["val_type"][k]), v0=int(pre["val0"][k]),
                     v1=int(pre["val1"][k]), ln=int(pre["val_len"][k]), site=int(pre["site"][k]),
                     dbv=int(pre["db_version"][k]), seq=int(pre["seq"][k]), pos=-1)
            rows.setdefault((c["table"], c["pk"]), []).append(c)
    vt = batch.get("val_type")
    for i in range(n):
        tc = int(batch["table_cid"][i])
        c = dict(pk=int(batch["pk"][i]), table=tc >> 16, cid=tc & 0xFFFF, cl=int(batch["cl"][i]),
                 cv=int(batch["col_version"][i]), t=int(vt[i]) if vt is not None else 1, v0=int(batch["val0"][i]),
                 v1=int(batch["val1"][i]) if "val1" in batch else 0,
                 ln=int(batch["val_len"][i]) if "val_len" in batch else 0, site=int(batch["site"][i]),
                 dbv=int(batch["db_version"][i]), seq=int(batch["seq"][i]), pos=i)
        rows.setdefault((c["table"], c["pk"]), []).append(c)
    got_rows, imp = [], np.zeros(n, np.uint8)
    fallback = 0
    for (t, pk), chs in rows.items():
        res = fold_row(chs)
        if res is None:
            fallback += 1
            continue
        rr, ii = res
        for c, v in zip(chs, ii):
            if c["pos"] >= 0:
                imp[c["pos"]] = v
        for x in rr:
            got_rows.append((t, pk, x["cid"], x["cv"], x["dbv"], x["site"], x["rowcl"], x["seq"], x["t"], x["v0"]))
    bad_rows = {(int(r[0]), int(r[1])) for r in []}
    ref_rows = []
    fb_keys = set()
    for (t, pk), chs in rows.items():
        if fold_row(chs) is None:
            fb_keys.add((t, pk))
    for k in range(len(ref["pk"])):
        tc = int(ref["table_cid"][k])
        if (tc >> 16, int(ref["pk"][k])) in fb_keys:
            continue
        ref_rows.append((tc >> 16, int(ref["pk"][k]), tc & 0xFFFF, int(ref["col_version"][k]),
                         int(ref["db_version"][k]), int(ref["site"][k]), int(ref["cl"][k]), int(ref["seq"][k]),
                         int(ref["val_type"][k]), int(ref["val0"][k])))
    fb_pos = [c["pos"] for (t, pk), chs in rows.items() if (t, pk) in fb_keys for c in chs if c["pos"] >= 0]
    mask = np.ones(n, bool)
    mask[fb_pos] = False
    ok_rows = sorted(got_rows) == sorted(ref_rows)
    ok_imp = np.array_equal(imp[mask], np.asarray(imp_ref)[mask])
    del bad_rows
    return ok_rows, ok_imp, fallback, len(rows)


def main():
    import synth
    tot = [0, 0, 0]
    for seed in range(60):
        sites = synth.site_ids(6, seed)
        for malformed in (False, True):
            b = synth.adversarial_batch(3000, 6, 2, 60 if seed % 2 else 400, seed, malformed=malformed,
                                        zipf=1.1 if seed % 3 else 0)
            prior = None
            if seed % 4 == 0:
                prior = synth.adversarial_batch(2000, 6, 2, 60 if seed % 2 else 400, seed + 1000, malformed=False)
            ok_rows, ok_imp, fb, nrows = check(b, sites, prior)
            tot[0] += 1
            tot[1] += ok_rows and ok_imp
            tot[2] += fb
            if not (ok_rows and ok_imp):
                print("MISMATCH seed", seed, "malformed", malformed, "rows", ok_rows, "impacts", ok_imp)
    print(f"{tot[1]}/{tot[0]} batches match; {tot[2]} rows fell back to the sequential fold")


if __name__ == "__main__":
    main()
