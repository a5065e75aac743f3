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
