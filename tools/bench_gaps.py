"""Batched gap bookkeeping on the device (corro_booked_insert_db_batch) at the config-4 universe
(VERDICT r1 item 9): 100k actors, each with 200 single-version gaps below max 599 (every third
version missing) and Poisson(2)+1 applied version ranges in [1, 700) this call -- the shape
tools/time_bookkeeping.py times on the host (~32 us per actor there). Prints one JSON line."""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import corrosion_amd as ca
    import corrosion_amd._lib as L
    from corrosion_amd.bookkeeping import canonical_ranges
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
    rng = np.random.default_rng(4)
    dev = torch.device("cuda", 0)
    # gaps: [3j, 3j] for j = 1..199, max 599
    g = np.arange(3, 600, 3, dtype=np.uint64)
    G1 = len(g)
    gap_off = np.arange(n + 1, dtype=np.uint64) * G1
    gs = np.tile(g, n)
    vers = []
    for _ in range(n):
        k = int(rng.poisson(2)) + 1
        st = rng.integers(1, 700, size=k)
        vers.append(canonical_ranges([(int(s), int(s + rng.integers(0, 20))) for s in st]))
    ver_off = np.zeros(n + 1, np.uint64)
    ver_off[1:] = np.cumsum([len(v) for v in vers])
    vs = np.array([r[0] for v in vers for r in v], np.uint64)
    ve = np.array([r[1] for v in vers for r in v], np.uint64)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)
    t = {"max": torch.full((n,), 599, dtype=torch.int64, device=dev), "gap_off": T(gap_off), "gap_start": T(gs),
         "gap_end": T(gs), "ver_off": T(ver_off), "ver_start": T(vs), "ver_end": T(ve)}
    G, V = int(gap_off[-1]), int(ver_off[-1])
    W = G + V + n
    o = {k: torch.empty(sz, dtype=torch.int64, device=dev) for k, sz in
         (("max", n), ("rm_count", n), ("ins_count", n), ("gap_count", n), ("rm_start", G), ("rm_end", G),
          ("ins_start", W), ("ins_end", W), ("new_start", W), ("new_end", W))}
    o["status"] = torch.empty(n, dtype=torch.int32, device=dev)
    eng = ca.MergeEngine({"t": ["a"]}, capacity_hint=1024)
    gi, go = L.GapsIn(), L.GapsOut()
    gi.n = n
    for k in t:
        setattr(gi, k, t[k].data_ptr())
    for k in o:
        setattr(go, k, o[k].data_ptr())
    torch.cuda.synchronize()
    eng.set_profiling(True)
    lib = L.lib()
    ms = []
    for it in range(8):
        L.check(lib.corro_booked_insert_db_batch(eng._h, C.byref(gi), C.byref(go)))
        if it >= 3:
            ms.append(eng.last_timings(apply_only=False)["k_needs_count"])
    ms.sort()
    k_ms = ms[len(ms) // 2]
    assert int((o["status"] != 0).sum()) == 0
    rows = int(o["rm_count"].sum() + o["ins_count"].sum())
    in_bytes = 16 * (G + V) + 8 * 3 * n
    out_bytes = 16 * (rows + int(o["gap_count"].sum())) + 8 * 4 * n
    print(json.dumps({"metric": "batched insert_db: actors/s", "value": n / (k_ms * 1e-3), "unit": "actors/s",
                      "actors": n, "kernel_ms": k_ms, "us_per_actor": k_ms * 1e3 / n,
                      "gap_rows_out": rows, "gaps_in": G, "version_ranges_in": V,
                      "roofline": {"bound": "hbm", "achieved": (in_bytes + out_bytes) / (k_ms * 1e-3) / 1e9,
                                   "peak": 8000.0, "unit": "GB/s"},
                      "host_reference": "tools/time_bookkeeping.py shape C: ~32 us per actor (host C++ insert_db)"}),
          flush=True)


if __name__ == "__main__":
    main()
