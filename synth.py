"""Seeded synthetic changesets for the BASELINE.json configs (SURVEY.md §8(d) "Concrete inputs").

All batches are SoA dicts in application order (actors ascending by 16-byte id, then version, then
seq — util.rs:705,765,782,1222). numpy variants feed tests and the CPU baseline; the torch variant
builds config 2 directly in HBM for bench.py.
"""
import numpy as np

MASK64 = (1 << 64) - 1


def splitmix64(x):
    x = (x + 0x9E3779B97F4A7C15) & MASK64
    z = x
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK64
    return z ^ (z >> 31)


def config_seed(cfg):
    return splitmix64(0xC0DE0000 + cfg)


def site_ids(n, seed):
    """n distinct random 16-byte actor ids, sorted ascending (ordinal == rank)."""
    rng = np.random.default_rng(seed)
    ids = rng.integers(0, 256, size=(n, 16), dtype=np.uint8)
    ids = np.unique(ids, axis=0)
    while ids.shape[0] < n:
        extra = rng.integers(0, 256, size=(n - ids.shape[0], 16), dtype=np.uint8)
        ids = np.unique(np.concatenate([ids, extra]), axis=0)
    return ids[:n]


def uniform_batch(n, nactors, npk, ncols, seed, cv_max=8, tie_frac=0.125, per_version=64, table=0,
                  pk_base=1):
    """Config 1/2 shape: cl = 1, INTEGER values, pk uniform in [pk_base, pk_base+npk)."""
    rng = np.random.default_rng(seed)
    per_actor = -(-n // nactors)
    i = np.arange(n, dtype=np.int64)
    site = (i // per_actor).astype(np.uint32)
    local = i % per_actor
    dbv = (local // per_version + 1).astype(np.int64)
    seq = (local % per_version).astype(np.uint32)
    pk = (rng.integers(0, npk, size=n, dtype=np.int64) + pk_base).astype(np.uint64)
    cid = rng.integers(1, ncols + 1, size=n, dtype=np.int64)
    tcid = ((table << 16) | cid).astype(np.uint32)
    cv = rng.integers(1, cv_max + 1, size=n, dtype=np.int64)
    val = rng.integers(-(1 << 62), 1 << 62, size=n, dtype=np.int64)
    ties = rng.random(n) < tie_frac
    val[ties] = rng.integers(0, 8, size=int(ties.sum()), dtype=np.int64)
    return {"pk": pk, "table_cid": tcid, "col_version": cv, "db_version": dbv,
            "cl": np.ones(n, np.uint32), "seq": seq, "site": site, "val0": val.view(np.uint64)}


def _zipf_pk(rng, n, npk, s):
    # bounded Zipf over [1, npk] by inverse CDF on a table
    ranks = np.arange(1, npk + 1, dtype=np.float64)
    w = ranks ** (-s)
    cdf = np.cumsum(w)
    cdf /= cdf[-1]
    u = rng.random(n)
    return (np.searchsorted(cdf, u) + 1).astype(np.uint64)


def adversarial_batch(n, nactors, ntables, npk, seed, zipf=1.1, sentinel_frac=0.3, wide=True,
                      malformed=False, per_version=50, max_cl=6):
    """Config 5 shape (scaled): Zipf pks, deletes/resurrects, mixed INTEGER + 16-byte BLOB columns.

    Schema per table: (id INTEGER PK, i0 INTEGER, i1 INTEGER, b0 BLOB, b1 BLOB) -> cids 1..4.
    Well-formed unless malformed=True: sentinel changes carry col_version == cl and
    NULL; column changes carry odd cl. With wide=True some values are REAL/TEXT/NULL too."""
    rng = np.random.default_rng(seed)
    per_actor = -(-n // nactors)
    i = np.arange(n, dtype=np.int64)
    site = (i // per_actor).astype(np.uint32)
    local = i % per_actor
    dbv = (local // per_version + 1).astype(np.int64)
    seq = (local % per_version).astype(np.uint32)
    table = rng.integers(0, ntables, size=n, dtype=np.int64)
    pk = _zipf_pk(rng, n, npk, zipf) if zipf else rng.integers(1, npk + 1, size=n).astype(np.uint64)
    sent = rng.random(n) < sentinel_frac
    cid = np.where(sent, 0, rng.integers(1, 5, size=n, dtype=np.int64))
    cl = rng.integers(1, max_cl + 1, size=n, dtype=np.int64)
    if not malformed:
        cl = np.where(sent, cl, cl | 1)  # column changes: odd causal length
    cv = rng.integers(1, 6, size=n, dtype=np.int64)
    if not malformed:
        cv = np.where(sent, cl, cv)
    vt = np.full(n, 1, np.uint8)
    v0 = rng.integers(-(1 << 62), 1 << 62, size=n, dtype=np.int64).view(np.uint64)
    ties = rng.random(n) < 0.3
    v0[ties] = rng.integers(0, 4, size=int(ties.sum())).astype(np.uint64)
    v1 = np.zeros(n, np.uint64)
    vl = np.zeros(n, np.uint8)
    blob = (cid == 3) | (cid == 4)
    vt[blob] = 4
    vl[blob] = 16
    v1[blob] = rng.integers(0, 1 << 63, size=int(blob.sum()), dtype=np.int64).astype(np.uint64)
    bt = blob & (rng.random(n) < 0.3)
    v1[bt] = rng.integers(0, 3, size=int(bt.sum())).astype(np.uint64)
    v0[bt] = rng.integers(0, 3, size=int(bt.sum())).astype(np.uint64)
    if wide:
        r = rng.random(n)
        real = (~blob) & (r < 0.1)
        vt[real] = 2
        v0[real] = rng.choice(np.array([0.0, -0.0, 1.5, -2.25, 5.0], np.float64), size=int(real.sum())).view(np.uint64)
        text = (~blob) & (r >= 0.1) & (r < 0.2)
        vt[text] = 3
        lens = rng.integers(0, 17, size=int(text.sum()))
        vl[text] = lens
        raw = rng.integers(97, 100, size=(int(text.sum()), 16), dtype=np.uint8)
        for k in range(raw.shape[0]):
            raw[k, lens[k]:] = 0
        v0[text] = raw[:, :8].copy().view(">u8").reshape(-1).astype(np.uint64)
        v1[text] = raw[:, 8:].copy().view(">u8").reshape(-1).astype(np.uint64)
        nul = (~blob) & (r >= 0.2) & (r < 0.25)
        vt[nul] = 5
        v0[nul] = 0
    vt[sent] = 5
    v0[sent] = 0
    v1[sent] = 0
    vl[sent] = 0
    tcid = ((table << 16) | cid).astype(np.uint32)
    return {"pk": pk, "table_cid": tcid, "col_version": cv.astype(np.int64), "db_version": dbv,
            "cl": cl.astype(np.uint32), "seq": seq, "site": site, "val0": v0, "val1": v1,
            "val_type": vt, "val_len": vl, "ts": (dbv.astype(np.uint64) << np.uint64(20)) + site.astype(np.uint64)}


def adversarial_batch_torch(n, nactors, ntables, npk, seed, device="cuda", zipf=1.1, sentinel_frac=0.3,
                            per_version=50, max_cl=6):
    """Config 5 generated in HBM (torch): the distribution of adversarial_batch(wide=True), not its
    bytes (bench.py's config-5 figure; parity tests use the numpy batch). Zipf pks by inverse CDF,
    30 % sentinels (col_version == cl, NULL), column changes at odd cl with INTEGER / 16-B BLOB /
    REAL / TEXT (<= 16 B inline) / NULL values."""
    import torch
    g = torch.Generator(device=device)
    g.manual_seed(seed & 0x7FFFFFFFFFFFFFFF)
    i64 = torch.int64
    per_actor = -(-n // nactors)
    i = torch.arange(n, device=device, dtype=i64)
    site = (i // per_actor).to(torch.int32)
    local = i % per_actor
    dbv = local // per_version + 1
    seq = (local % per_version).to(torch.int32)
    table = torch.randint(0, ntables, (n,), device=device, generator=g, dtype=i64)
    w = torch.arange(1, npk + 1, device=device, dtype=torch.float64) ** (-zipf)
    cdf = torch.cumsum(w, 0)
    cdf /= cdf[-1].clone()
    pk = (torch.searchsorted(cdf, torch.rand(n, device=device, generator=g, dtype=torch.float64)) + 1).clamp(max=npk)
    sent = torch.rand(n, device=device, generator=g) < sentinel_frac
    cid = torch.where(sent, torch.zeros_like(table), torch.randint(1, 5, (n,), device=device, generator=g, dtype=i64))
    cl = torch.randint(1, max_cl + 1, (n,), device=device, generator=g, dtype=i64)
    cl = torch.where(sent, cl, cl | 1)
    cv = torch.where(sent, cl, torch.randint(1, 6, (n,), device=device, generator=g, dtype=i64))
    vt = torch.ones(n, device=device, dtype=torch.uint8)
    v0 = torch.randint(-(1 << 62), 1 << 62, (n,), device=device, generator=g, dtype=i64)
    ties = torch.rand(n, device=device, generator=g) < 0.3
    v0 = torch.where(ties, torch.randint(0, 4, (n,), device=device, generator=g, dtype=i64), v0)
    v1 = torch.zeros(n, device=device, dtype=i64)
    vl = torch.zeros(n, device=device, dtype=torch.uint8)
    blob = (cid == 3) | (cid == 4)
    vt = torch.where(blob, torch.full_like(vt, 4), vt)
    vl = torch.where(blob, torch.full_like(vl, 16), vl)
    v1 = torch.where(blob, torch.randint(0, 1 << 62, (n,), device=device, generator=g, dtype=i64), v1)
    bt = blob & (torch.rand(n, device=device, generator=g) < 0.3)
    v1 = torch.where(bt, torch.randint(0, 3, (n,), device=device, generator=g, dtype=i64), v1)
    v0 = torch.where(bt, torch.randint(0, 3, (n,), device=device, generator=g, dtype=i64), v0)
    r = torch.rand(n, device=device, generator=g)
    real = (~blob) & (r < 0.1)
    reals = torch.tensor([0.0, -0.0, 1.5, -2.25, 5.0], device=device, dtype=torch.float64).view(i64)
    v0 = torch.where(real, reals[torch.randint(0, 5, (n,), device=device, generator=g)], v0)
    vt = torch.where(real, torch.full_like(vt, 2), vt)
    text = (~blob) & (r >= 0.1) & (r < 0.2)
    lens = torch.randint(0, 17, (n,), device=device, generator=g, dtype=i64)
    raw = torch.randint(97, 100, (n, 16), device=device, generator=g, dtype=i64)
    raw = torch.where(torch.arange(16, device=device)[None, :] < lens[:, None], raw, torch.zeros_like(raw))
    sh = (8 * (7 - torch.arange(8, device=device, dtype=i64)))[None, :]
    tw0 = (raw[:, :8] << sh).sum(1)
    tw1 = (raw[:, 8:] << sh).sum(1)
    del raw
    v0 = torch.where(text, tw0, v0)
    v1 = torch.where(text, tw1, v1)
    vt = torch.where(text, torch.full_like(vt, 3), vt)
    vl = torch.where(text, lens.to(torch.uint8), vl)
    nul = (~blob) & (r >= 0.2) & (r < 0.25)
    vt = torch.where(nul, torch.full_like(vt, 5), vt)
    v0 = torch.where(nul, torch.zeros_like(v0), v0)
    vt = torch.where(sent, torch.full_like(vt, 5), vt)
    zero = torch.zeros_like(v0)
    v0, v1 = torch.where(sent, zero, v0), torch.where(sent, zero, v1)
    vl = torch.where(sent, torch.zeros_like(vl), vl)
    tcid = ((table << 16) | cid).to(torch.int32)
    return {"pk": pk.contiguous(), "table_cid": tcid.contiguous(), "col_version": cv.contiguous(),
            "db_version": dbv.contiguous(), "cl": cl.to(torch.int32).contiguous(), "seq": seq.contiguous(),
            "site": site.contiguous(), "val0": v0.contiguous(), "val1": v1.contiguous(),
            "val_type": vt.contiguous(), "val_len": vl.contiguous(), "ts": ((dbv << 20) + site.to(i64)).contiguous()}


def blob_pks_torch(ids, device="cuda"):
    """testsblob-shaped packed pks (pack_columns of one 16-byte BLOB, corro-tests/src/lib.rs:32-35)
    generated in HBM from integer row ids: 19 bytes each -- column count 1, type byte (1 << 3 | BLOB),
    length 16, then the id big-endian and a 64-bit mix of it -- so distinct ids are distinct keys.
    Returns (uint8 bytes, int64 offsets of n + 1)."""
    import torch
    ids = ids.to(device=device, dtype=torch.int64)
    n = ids.numel()
    x = ids.clone()
    m = ids * -7046029254386353131 + 0x165667B19E3779F9  # (wrapping int64 arithmetic)
    m = m ^ ((m >> 29) & 0x7FFFFFFFF)
    out = torch.empty((n, 19), dtype=torch.uint8, device=device)
    out[:, 0] = 1
    out[:, 1] = (1 << 3) | 4
    out[:, 2] = 16
    for k in range(8):
        out[:, 3 + k] = ((x >> (8 * (7 - k))) & 0xFF).to(torch.uint8)
        out[:, 11 + k] = ((m >> (8 * (7 - k))) & 0xFF).to(torch.uint8)
    off = torch.arange(0, 19 * (n + 1), 19, dtype=torch.int64, device=device)
    return out.reshape(-1), off


ADV_COLS = ["i0", "i1", "b0", "b1"]


def adversarial_schema(ntables):
    return {f"t{k}": list(ADV_COLS) for k in range(ntables)}


def uniform_batch_torch(n, nactors, npk, ncols, seed, device="cuda", cv_max=8, per_version=64, offset=0,
                        global_n=None):
    """Config 2 generated in HBM (torch), same distribution as uniform_batch. `offset` / `global_n`
    generate the slice [offset, offset + n) of a global batch of global_n changes (config 3's
    rank-major batch: actors, versions and seqs numbered over the whole batch)."""
    import torch
    g = torch.Generator(device=device)
    g.manual_seed(seed & 0x7FFFFFFFFFFFFFFF)
    per_actor = -(-(global_n or n) // nactors)
    i = torch.arange(offset, offset + n, device=device, dtype=torch.int64)
    site = (i // per_actor).to(torch.int32)
    local = i % per_actor
    dbv = local // per_version + 1
    seq = (local % per_version).to(torch.int32)
    pk = torch.randint(0, npk, (n,), device=device, generator=g, dtype=torch.int64) + 1
    cid = torch.randint(1, ncols + 1, (n,), device=device, generator=g, dtype=torch.int64)
    cv = torch.randint(1, cv_max + 1, (n,), device=device, generator=g, dtype=torch.int64)
    val = torch.randint(-(1 << 62), 1 << 62, (n,), device=device, generator=g, dtype=torch.int64)
    ties = torch.rand(n, device=device, generator=g) < 0.125
    small = torch.randint(0, 8, (n,), device=device, generator=g, dtype=torch.int64)
    val = torch.where(ties, small, val)
    return {"pk": pk.contiguous(), "table_cid": cid.to(torch.int32).contiguous(), "col_version": cv.contiguous(),
            "db_version": dbv.contiguous(), "cl": torch.ones(n, device=device, dtype=torch.int32),
            "seq": seq.contiguous(), "site": site.contiguous(), "val0": val.contiguous()}


def sync_entries_torch(npairs, actors_per_pair, seed, device="cuda", max_head=1_000_000,
                       need_rate=2.0, need_len=20, partial_frac=0.05):
    """Config 4 generated in HBM: npairs node-pair states, each with
    `actors_per_pair` sparse actors -> one CSR entry per (pair, actor). Per side: head uniform in
    [1, max_head] (ours absent 10 %), Poisson(need_rate) disjoint non-adjacent need ranges of
    geometric length (mean need_len); 5 % of entries carry a partial version (1-3 seq ranges in
    [0, 1000]), half of them at the same version on both sides."""
    import torch
    g = torch.Generator(device=device)
    g.manual_seed(seed & 0x7FFFFFFFFFFFFFFF)
    E = npairs * actors_per_pair
    i64 = torch.int64

    def ranges(cnt, gap_mean, len_mean, base):
        R = int(cnt.sum().item())
        off = torch.zeros(E + 1, dtype=i64, device=device)
        off[1:] = torch.cumsum(cnt, 0)
        if R == 0:
            z = torch.zeros(0, dtype=i64, device=device)
            return off, z, z
        ent = torch.repeat_interleave(torch.arange(E, device=device), cnt)
        # (a float geometric sample can round to 0: clamp, so ranges are non-empty and non-adjacent as
        # generate_sync's RangeInclusiveSet gives them)
        gap = torch.empty(R, device=device).geometric_(1.0 / gap_mean, generator=g).to(i64).clamp(min=1) + 1
        ln = torch.empty(R, device=device).geometric_(1.0 / len_mean, generator=g).to(i64).clamp(min=1)
        step = gap + ln
        cs = torch.cumsum(step, 0)
        first = off[:-1][ent]
        prior = torch.where(first > 0, cs[(first - 1).clamp(min=0)], torch.zeros_like(first))
        seg = cs - prior                      # segmented inclusive cumsum per entry
        end = seg + base
        start = end - ln + 1
        return off, start, end

    their_head = torch.randint(1, max_head + 1, (E,), device=device, generator=g)
    our_head = torch.randint(1, max_head + 1, (E,), device=device, generator=g)
    our_head = torch.where(torch.rand(E, device=device, generator=g) < 0.1, torch.full_like(our_head, -1), our_head)
    tn_cnt = torch.poisson(torch.full((E,), need_rate, device=device), generator=g).to(i64)
    on_cnt = torch.poisson(torch.full((E,), need_rate, device=device), generator=g).to(i64)
    span = max(1, max_head // 20)
    tn_off, tn_s, tn_e = ranges(tn_cnt, span // 4 + 2, need_len, 0)
    on_off, on_s, on_e = ranges(on_cnt, span // 4 + 2, need_len, 0)

    def partials(shared_ver):
        has = torch.rand(E, device=device, generator=g) < partial_frac
        cnt = has.to(i64)
        off = torch.zeros(E + 1, dtype=i64, device=device)
        off[1:] = torch.cumsum(cnt, 0)
        ids = torch.nonzero(has).flatten()
        ver = torch.where(torch.rand(ids.numel(), device=device, generator=g) < 0.5, shared_ver[ids],
                          (torch.rand(ids.numel(), device=device, generator=g) * their_head[ids]).to(i64) + 1)
        scnt = torch.randint(1, 4, (ids.numel(),), device=device, generator=g)
        soff = torch.zeros(ids.numel() + 1, dtype=i64, device=device)
        soff[1:] = torch.cumsum(scnt, 0)
        S = int(soff[-1].item())
        pid = torch.repeat_interleave(torch.arange(ids.numel(), device=device), scnt)
        gap = torch.randint(0, 200, (S,), device=device, generator=g) + 2
        ln = torch.randint(0, 150, (S,), device=device, generator=g)
        cs = torch.cumsum(gap + ln, 0)
        first = soff[:-1][pid]
        prior = torch.where(first > 0, cs[(first - 1).clamp(min=0)], torch.zeros_like(first))
        e_ = cs - prior
        return off, ver, soff, e_ - ln, e_

    shared = (torch.rand(E, device=device, generator=g) * their_head).to(i64) + 1
    tp_off, tp_ver, tps_off, tps_s, tps_e = partials(shared)
    op_off, op_ver, ops_off, ops_s, ops_e = partials(shared)
    return {"their_head": their_head, "our_head": our_head, "tn_off": tn_off, "tn_start": tn_s, "tn_end": tn_e,
            "tp_off": tp_off, "tp_ver": tp_ver, "tps_off": tps_off, "tps_start": tps_s, "tps_end": tps_e,
            "on_off": on_off, "on_start": on_s, "on_end": on_e, "op_off": op_off, "op_ver": op_ver,
            "ops_off": ops_off, "ops_start": ops_s, "ops_end": ops_e}


# long TEXT/BLOB values (> 16 bytes) that tie on their first 8 / 16 bytes, differ only past them, or
# only in length -- the cases a prefix compare would get wrong
LONG_POOL = [b"hello world, this is a long value", b"hello world, this is a long valuf",
             b"hello world, this is a long value!", b"0123456789abcdef0", b"0123456789abcdef" * 9,
             b"\0" * 17, b"\0" * 40, b"\0" * 16 + b"\1", bytes(range(200)), b"aaaaaaaaaaaaaaaaaaaaaaaaa"]


def with_long_values(b, seed, frac=0.2, pool=LONG_POOL):
    """A copy of batch b in which about `frac` of the column changes carry a long TEXT/BLOB value
    (val_len 255, bytes in val_data at val_off / val_size)."""
    rng = np.random.default_rng(seed)
    n = len(b["pk"])
    out = dict(b)
    vt = np.array(b.get("val_type", np.ones(n, np.uint8)), np.uint8, copy=True)
    vl = np.array(b.get("val_len", np.zeros(n, np.uint8)), np.uint8, copy=True)
    v0 = np.array(b["val0"], np.uint64, copy=True)
    v1 = np.array(b.get("val1", np.zeros(n, np.uint64)), np.uint64, copy=True)
    pick = ((np.asarray(b["table_cid"]) & 0xFFFF) != 0) & (rng.random(n) < frac)
    which = rng.integers(0, len(pool), size=n)
    off, size = np.zeros(n, np.uint64), np.zeros(n, np.uint32)
    data, dlen = [], 0
    for i in np.nonzero(pick)[0]:
        v = pool[which[i]]
        vt[i] = 3 if (which[i] % 2 == 0) else 4
        vl[i] = 255
        v0[i] = int.from_bytes(v[:8], "big")
        v1[i] = 0
        off[i], size[i] = dlen, len(v)
        data.append(v)
        dlen += len(v)
    out.update({"val_type": vt, "val_len": vl, "val0": v0, "val1": v1, "val_off": off, "val_size": size,
                "val_data": np.frombuffer(b"".join(data) or b"\0", np.uint8)[:dlen]})
    return out
