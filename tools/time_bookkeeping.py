"""Host cost of the gap bookkeeping (VersionsSnapshot::insert_db, agent.rs:1108-1235) at the sizes of
the merge workloads, to place it against the device apply. Calls
corro_booked_insert_db directly through ctypes with preallocated buffers (no Python per range).

  A  config-2 shape: one process_multiple_changes of 2^26 changes = 1000 actors x 1049 versions of
     64 changes, each actor's versions arriving in order (one coalesced range per actor per call)
  B  the same versions arriving as 8 interleaved batches with holes (gaps opened, then closed)
  C  config-4 universe: 100k actors, each call bringing Poisson(2)+1 ranges per actor with random
     holes against a state already holding gaps (the sync-heavy shape)
Prints one JSON line; CPU only (the bookkeeping is host C++)."""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import corrosion_amd._lib as L
    lib = L.lib()
    cap = 1 << 16
    bufs = [np.zeros(cap, np.uint64) for _ in range(4)]
    nr, ni = C.c_uint64(), C.c_uint64()

    def new():
        h = C.c_void_p()
        L.check(lib.corro_booked_new(C.byref(h)))
        return h

    def insert(h, s, e):
        L.check(lib.corro_booked_insert_db(h, s.ctypes.data, e.ctypes.data, len(s), bufs[0].ctypes.data,
                                           bufs[1].ctypes.data, cap, C.byref(nr), bufs[2].ctypes.data,
                                           bufs[3].ctypes.data, cap, C.byref(ni)))
        return nr.value + ni.value

    out = {}
    # A: 1000 actors, versions 1..1049 as one range each
    hs = [new() for _ in range(1000)]
    t0 = time.perf_counter()
    for h in hs:
        insert(h, np.array([1], np.uint64), np.array([1049], np.uint64))
    out["A_one_call_1000_actors_ms"] = (time.perf_counter() - t0) * 1e3
    # B: 8 batches, batch j brings versions v with v % 8 == j (holes everywhere until the last)
    hs = [new() for _ in range(1000)]
    rows = 0
    t0 = time.perf_counter()
    for j in range(8):
        v = np.arange(1 + j, 1050, 8, dtype=np.uint64)
        for h in hs:
            rows += insert(h, v, v)
    dt = time.perf_counter() - t0
    out["B_8_interleaved_calls_1000_actors_ms_per_call"] = dt * 1e3 / 8
    out["B_gap_rows_per_call"] = rows / 8
    # C: 100k actors, existing gaps, Poisson(2)+1 ranges per actor per call
    rng = np.random.default_rng(4)
    hs = [new() for _ in range(100_000)]
    for h in hs:  # initial state with holes: every 3rd of 1..600 missing
        v = np.arange(1, 601, dtype=np.uint64)
        v = v[v % 3 != 0]
        insert(h, v, v)
    calls = []
    for h in hs:
        k = int(rng.poisson(2)) + 1
        st = np.sort(rng.integers(1, 700, size=k)).astype(np.uint64)
        calls.append((st, st + rng.integers(0, 20, size=k).astype(np.uint64)))
    t0 = time.perf_counter()
    rows = 0
    for h, (s, e) in zip(hs, calls):
        rows += insert(h, s, e)
    dt = time.perf_counter() - t0
    out["C_one_call_100k_actors_ms"] = dt * 1e3
    out["C_us_per_actor"] = dt * 1e6 / len(hs)
    out["C_gap_rows"] = rows
    out["note"] = ("host C++ insert_db through ctypes (~0.3-0.5 us of each call is the ctypes crossing); "
                   "compare with the device apply of the same call: config 2 (2^26 changes) 3.7 ms")
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
