"""corro_process_multiple_changes with many actors (the batched gap bookkeeping route).

100 K actors (ACTORS) x 8 versions x 8 changes arrive in a first call with versions 3 and 6 missing
(two gaps per actor), then a second call fills both gaps and adds versions 9-10 (HOLES=h: the odd
versions below 2h first, the even ones second). The second call is
timed with the per-actor host insert_db (CORRO_AGENT_GAPS_BATCH=0) and with the batched device
pass (=1); headers, changes and outcomes in HBM (CORRO_MEM_DEVICE_HEADERS), fresh Bookie and
state per rep, the first call untimed. Prints one JSON line."""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

N_ACT = int(os.environ.get("ACTORS", "100000"))
PER = 8


def build(versions, ids, rng, dev):
    import torch
    from corrosion_amd import _lib as L
    cs_dt = np.dtype([("actor_id", "<u8"), ("site", "<u4"), ("kind", "<u4"), ("version_start", "<u8"),
                      ("version_end", "<u8"), ("seq_start", "<u8"), ("seq_end", "<u8"), ("last_seq", "<u8"),
                      ("ts", "<u8"), ("change_off", "<u8"), ("change_count", "<u8")])
    a_idx = np.tile(np.arange(N_ACT, dtype=np.int64), len(versions))      # arrival: round-robin by version
    v_idx = np.repeat(np.asarray(versions, dtype=np.int64), N_ACT)
    ncs = len(a_idx)
    cs = np.zeros(ncs, cs_dt)
    cs["actor_id"] = ids.ctypes.data + 16 * a_idx
    cs["site"] = a_idx
    cs["kind"] = L.CORRO_CS_FULL
    cs["version_start"] = cs["version_end"] = v_idx
    cs["seq_end"] = cs["last_seq"] = PER - 1
    cs["ts"] = (v_idx << 32) | a_idx
    cs["change_off"] = np.arange(ncs, dtype=np.int64) * PER
    cs["change_count"] = PER
    n = ncs * PER
    g = torch.Generator(device=dev)
    g.manual_seed(int(rng.integers(1 << 30)))
    rep = lambda x: torch.from_numpy(np.repeat(x, PER)).to(dev)
    batch = {
        "pk": torch.randint(1, 1 << 22, (n,), device=dev, generator=g, dtype=torch.int64),
        "table_cid": torch.randint(1, 5, (n,), device=dev, generator=g, dtype=torch.int32),
        "col_version": torch.randint(1, 8, (n,), device=dev, generator=g, dtype=torch.int64),
        "db_version": rep(v_idx),
        "cl": torch.ones(n, dtype=torch.int32, device=dev),
        "seq": torch.arange(PER, dtype=torch.int32, device=dev).repeat(ncs),
        "site": rep(a_idx.astype(np.int32)),
        "val0": torch.randint(0, 1 << 40, (n,), device=dev, generator=g, dtype=torch.int64),
        "ts": rep((v_idx << 32) | a_idx),
    }
    return cs, batch, n


def call(eng, bk, cs_t, ncs, batch, n, known, imp):
    from corrosion_amd import _lib as L
    s = L.Changes()
    s.n = n
    for k, t in batch.items():
        setattr(s, k, t.data_ptr())
    out = L.ProcessOut()
    out.known, out.impactful = known.data_ptr(), imp.data_ptr()
    L.check(L.lib().corro_process_multiple_changes(eng._h, bk._h, C.c_void_p(cs_t.data_ptr()), ncs, C.byref(s),
                                                   L.CORRO_MEM_DEVICE_HEADERS, C.byref(out)))


def main():
    import torch
    import synth
    import corrosion_amd as ca
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(7)
    id_list = synth.site_ids(N_ACT, 3)
    ids = np.ascontiguousarray(id_list, dtype=np.uint8)
    eng = ca.MergeEngine({"t": ["a", "b", "c", "d"]}, capacity_hint=1 << 24)
    eng.register_sites(id_list)
    holes = int(os.environ.get("HOLES", "0"))  # >0: odd versions 1..2*HOLES-1 first (HOLES-1 gaps), then the even ones
    if holes:
        first = list(range(1, 2 * holes, 2))
        second = list(range(2, 2 * holes + 1, 2))
    else:
        first = [v for v in range(1, PER + 1) if v not in (3, 6)]
        second = [3, 6, 9, 10]
    cs1, b1, n1 = build(first, ids, rng, dev)
    cs2, b2, n2 = build(second, ids, rng, dev)
    t1 = torch.from_numpy(cs1.view(np.uint8).copy()).to(dev)
    t2 = torch.from_numpy(cs2.view(np.uint8).copy()).to(dev)
    k1 = torch.zeros(len(cs1), dtype=torch.int32, device=dev)
    k2 = torch.zeros(len(cs2), dtype=torch.int32, device=dev)
    i1 = torch.zeros(n1, dtype=torch.uint8, device=dev)
    i2 = torch.zeros(n2, dtype=torch.uint8, device=dev)
    res = {}
    for mode in ("0", "1", "0", "1"):
        os.environ["CORRO_AGENT_GAPS_BATCH"] = mode
        ms = []
        for _ in range(3):
            bk = ca.agent.Bookie()
            eng.reset()
            call(eng, bk, t1, len(cs1), b1, n1, k1, i1)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            call(eng, bk, t2, len(cs2), b2, n2, k2, i2)
            torch.cuda.synchronize()
            ms.append((time.perf_counter() - t0) * 1e3)
            gaps = sum(len(bk.needed(bytes(ids[a]))) for a in range(0, N_ACT, max(1, N_ACT // 1000)))
            del bk
        ms.sort()
        res.setdefault(mode, []).append(ms[1])
    print(json.dumps({"actors": N_ACT, "holes": holes, "changes_second_call": n2, "changesets_second_call": len(cs2),
                      "host_insert_db_ms": min(res["0"]), "device_batch_ms": min(res["1"]),
                      "gaps_left_sampled": gaps,
                      "note": "second call of a pair (HOLES=0: fills two gaps per actor and adds two versions; "
                              "HOLES=h: the first call leaves h-1 gaps per actor, the second fills them all); "
                              "CORRO_AGENT_GAPS_BATCH=0 (per-actor host insert_db) vs 1 (one device pass)"}),
          flush=True)


if __name__ == "__main__":
    main()
