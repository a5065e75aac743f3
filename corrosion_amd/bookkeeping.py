"""BookedVersions mirror (gap bookkeeping), backed by the C++ implementation in csrc/booked.cpp.

Mirrors /root/reference/crates/corro-types/src/agent.rs: VersionsSnapshot::insert_db (:1108-1168),
compute_gaps_change (:1170-1235), BookedVersions::{contains_version :1353, contains_all :1384,
last :1392}.
"""
import ctypes as C

import numpy as np

from . import _lib as L


class BookedVersions:
    def __init__(self):
        h = C.c_void_p()
        L.check(L.lib().corro_booked_new(C.byref(h)))
        self._h = h

    def __del__(self):
        if getattr(self, "_h", None):
            L.lib().corro_booked_free(self._h)
            self._h = None

    def insert_db(self, ranges):
        """Apply version ranges; returns (removed gap rows, inserted gap rows) as lists of (s, e)
        mirroring the DELETE / INSERT statements on __corro_bookkeeping_gaps."""
        s = np.array([r[0] for r in ranges], np.uint64)
        e = np.array([r[1] for r in ranges], np.uint64)
        cap = 2 * len(ranges) + 8 + self.needed_len()
        rs, re_, is_, ie = (np.zeros(cap, np.uint64) for _ in range(4))
        nr, ni = C.c_uint64(), C.c_uint64()
        L.check(L.lib().corro_booked_insert_db(
            self._h, s.ctypes.data if len(s) else None, e.ctypes.data if len(e) else None, len(ranges),
            rs.ctypes.data, re_.ctypes.data, cap, C.byref(nr), is_.ctypes.data, ie.ctypes.data, cap,
            C.byref(ni)))
        assert nr.value <= cap and ni.value <= cap
        return ([(int(rs[i]), int(re_[i])) for i in range(nr.value)],
                [(int(is_[i]), int(ie[i])) for i in range(ni.value)])

    def needed_len(self):
        c = C.c_uint64()
        L.check(L.lib().corro_booked_needed(self._h, None, None, 0, C.byref(c)))
        return c.value

    def needed(self):
        m = self.needed_len()
        s = np.zeros(max(m, 1), np.uint64)
        e = np.zeros(max(m, 1), np.uint64)
        c = C.c_uint64()
        L.check(L.lib().corro_booked_needed(self._h, s.ctypes.data, e.ctypes.data, m, C.byref(c)))
        return [(int(s[i]), int(e[i])) for i in range(m)]

    def last(self):
        v = C.c_int64()
        L.check(L.lib().corro_booked_last(self._h, C.byref(v)))
        return None if v.value < 0 else v.value

    def contains_version(self, version):
        r = C.c_int()
        L.check(L.lib().corro_booked_contains(self._h, version, C.byref(r)))
        return bool(r.value)

    def contains_all(self, start, end):
        r = C.c_int()
        L.check(L.lib().corro_booked_contains_all(self._h, start, end, C.byref(r)))
        return bool(r.value)


def canonical_ranges(ranges):
    """RangeInclusiveSet of (s, e) pairs: sorted, overlapping and touching ranges coalesced."""
    out = []
    for s, e in sorted((int(s), int(e)) for s, e in ranges):
        if out and s <= out[-1][1] + 1:
            if e > out[-1][1]:
                out[-1][1] = e
        else:
            out.append([s, e])
    return [tuple(r) for r in out]


def insert_db_batch(engine, maxes, gaps, versions):
    """corro_booked_insert_db_batch for len(maxes) actors at once on the engine's device.
    maxes: per actor max or None; gaps / versions: per actor lists of (s, e) (versions are made a
    RangeInclusiveSet first, as insert_db's caller builds one). Returns per actor
    (max, removed rows, inserted rows, needed gaps, status)."""
    import torch
    lib = L.lib()
    n = len(maxes)
    dev = torch.device("cuda", engine.device) if hasattr(engine, "device") else torch.device("cuda")
    versions = [canonical_ranges(v) for v in versions]

    def csr(lists):
        off = np.zeros(n + 1, np.uint64)
        off[1:] = np.cumsum([len(x) for x in lists])
        flat = [r for x in lists for r in x]
        s = np.array([r[0] for r in flat], np.uint64)
        e = np.array([r[1] for r in flat], np.uint64)
        return off, s, e

    def to_dev(a, dtype=torch.int64):
        a = np.ascontiguousarray(a)
        return torch.from_numpy(a.view(np.int64) if a.dtype == np.uint64 else a).to(dev) if a.size else \
            torch.zeros(1, dtype=dtype, device=dev)

    goff, gs, ge = csr(gaps)
    voff, vs, ve = csr(versions)
    mx = np.array([-1 if m is None else int(m) for m in maxes], np.int64)
    G, V = int(goff[-1]), int(voff[-1])
    W = G + V + n
    t = {"max": to_dev(mx), "gap_off": to_dev(goff), "gap_start": to_dev(gs), "gap_end": to_dev(ge),
         "ver_off": to_dev(voff), "ver_start": to_dev(vs), "ver_end": to_dev(ve)}
    o = {k: torch.zeros(max(1, sz), dtype=dt, device=dev) for k, sz, dt in
         (("max", n, torch.int64), ("rm_count", n, torch.int64), ("ins_count", n, torch.int64),
          ("gap_count", n, torch.int64), ("rm_start", G, torch.int64), ("rm_end", G, torch.int64),
          ("ins_start", W, torch.int64), ("ins_end", W, torch.int64), ("new_start", W, torch.int64),
          ("new_end", W, torch.int64), ("status", n, torch.int32))}
    gi = L.GapsIn()
    gi.n = n
    for k in ("max", "gap_off", "gap_start", "gap_end", "ver_off", "ver_start", "ver_end"):
        setattr(gi, k, t[k].data_ptr())
    go = L.GapsOut()
    for k in o:
        setattr(go, k, o[k].data_ptr())
    torch.cuda.synchronize(dev)
    L.check(lib.corro_booked_insert_db_batch(engine._h, C.byref(gi), C.byref(go)))
    h = {k: v.cpu().numpy() for k, v in o.items()}
    res = []
    for a in range(n):
        rb, ib = int(goff[a]), int(goff[a] + voff[a]) + a
        nr, ni, ng = int(h["rm_count"][a]), int(h["ins_count"][a]), int(h["gap_count"][a])
        res.append((None if h["max"][a] < 0 else int(h["max"][a]),
                    [(int(h["rm_start"][rb + i]), int(h["rm_end"][rb + i])) for i in range(nr)],
                    [(int(h["ins_start"][ib + i]), int(h["ins_end"][ib + i])) for i in range(ni)],
                    [(int(h["new_start"][ib + i]), int(h["new_end"][ib + i])) for i in range(ng)],
                    int(h["status"][a])))
    return res
