"""CPU checks of the drop-in boundary: the C-ABI library loads, exports every symbol
include/corro_hip.h declares, and its host-side pieces (gap bookkeeping) match the reference KATs.
No compute call needs a GPU here; compute entry points must refuse to run without one."""
import os
import re

import pytest

import corrosion_amd as ca
from corrosion_amd import _lib as L
from tests._util import load_golden

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    src = open(os.path.join(ROOT, "include", "corro_hip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(corro_[a-z_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    lib = L.lib()
    syms = header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), s
    assert sorted(L.EXPORTS) == syms


def test_abi_version():
    assert L.lib().corro_abi_version() == 3


def test_no_cpu_fallback_without_device():
    if ca.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(ca.CorroError) as e:
        ca.MergeEngine({"t": ["a", "b", "c"]})
    assert e.value.code == -7  # CORRO_E_NO_DEVICE


def test_booked_gap_kats_product():
    """VersionsSnapshot::insert_db through the product C++ (agent.rs:1605-1868)."""
    steps = load_golden("gaps_kats.json")["steps"]
    b, allv = ca.BookedVersions(), []
    for st in steps:
        if st.get("reset"):
            b, allv = ca.BookedVersions(), []
            continue
        b.insert_db([tuple(r) for r in st["insert"]])
        allv += st["insert"]
        if st["gaps"] is not None:
            assert b.needed() == [tuple(g) for g in st["gaps"]]
            for s, e in st["gaps"]:
                assert not b.contains_all(s, e)
                for v in range(s, e + 1):
                    assert not b.contains_version(v)
        assert b.last() == max(e for _, e in allv)
    # every inserted range is known at the end (expect_gaps: contains_all over all versions)
    for s, e in allv:
        gaps = [tuple(g) for g in steps[-1]["gaps"]]
        for v in range(s, e + 1):
            if not any(a <= v <= z for a, z in gaps):
                assert b.contains_version(v)


def test_booked_reports_gap_row_changes():
    """insert_db returns exactly the __corro_bookkeeping_gaps DELETE/INSERT rows."""
    b = ca.BookedVersions()
    assert b.insert_db([(1, 1), (4, 4)]) == ([], [(2, 3)])
    assert b.insert_db([(3, 3)]) == ([(2, 3)], [(2, 2)])
    assert b.insert_db([(2, 2)]) == ([(2, 2)], [])
    assert b.needed() == []


def test_booked_matches_oracle_random():
    from oracle import oracle as O
    import numpy as np
    rng = np.random.default_rng(7)
    for trial in range(200):
        p, o = ca.BookedVersions(), O.Booked()
        for step in range(int(rng.integers(1, 12))):
            k = int(rng.integers(1, 4))
            rs = []
            for _ in range(k):
                s = int(rng.integers(1, 60))
                rs.append((s, s + int(rng.integers(0, 6))))
            p.insert_db(rs)
            assert o.insert_db(rs) in (0, -1)
            assert p.needed() == o.needed(), (trial, step)
            assert p.last() == o.max()
            for v in range(1, 70):
                assert p.contains_version(v) == o.contains(v)


def _canon(b):
    import ctypes as C
    out = (C.c_uint8 * 256)()
    n = C.c_uint64()
    rc = L.lib().corro_pk_canonical(bytes(b), len(b), out, 256, C.byref(n))
    return None if rc else bytes(out[:n.value])


def test_pk_canonical_form():
    """pack_columns / unpack_columns (pubsub.rs:2304-2451) round trip, quirks included: integers in the
    fewest bytes num_bytes_needed_i64 gives (0 -> no bytes, negatives -> 8), TEXT/BLOB length in
    num_bytes_needed_i32 bytes; a non-canonical encoding of one key canonicalises to the same bytes."""
    assert _canon(b"\x01\x09\x01") == b"\x01\x09\x01"                      # Integer(1)
    assert _canon(b"\x01\x01") == b"\x01\x01"                              # Integer(0): no int bytes
    assert _canon(b"\x01\x21\x00\x00\x00\x01") == b"\x01\x09\x01"          # 1 in 4 bytes -> 1 byte
    assert _canon(b"\x01\x11\x01\x00") == b"\x01\x11\x01\x00"              # Integer(256): 2 bytes
    assert _canon(b"\x01\x09\xff") == b"\x01\x41" + b"\xff" * 8            # get_int sign-extends: -1 -> 8 bytes
    assert _canon(b"\x01\x0b\x02ab") == b"\x01\x0b\x02ab"                  # Text("ab")
    blob16 = bytes(range(16))
    assert _canon(b"\x01\x0c\x10" + blob16) == b"\x01\x0c\x10" + blob16    # Blob(16 bytes)
    comp = b"\x02\x0c\x08" + b"\x00" * 7 + b"\x05" + b"\x0b\x01" + b"5"      # (Blob(be 5), Text("5")): wide's pk
    assert _canon(comp) == comp
    assert _canon(b"\x01\x02" + b"\x80" + b"\x00" * 7) == b"\x01\x02" + b"\x00" * 8  # REAL -0.0 == 0.0
    assert _canon(b"\x01\x05") == b"\x01\x05"                              # NULL
    assert _canon(b"\x01\x0b\x05ab") is None                               # length past the end
    assert _canon(b"\x01\x07") is None                                     # no such column type


def test_affinity_of_type_rules():
    """sqlite3AffinityType's rule order (the column types of schema.rs): INT anywhere -> INTEGER
    (so 'FLOATING POINT' is INTEGER), CHAR/CLOB/TEXT -> TEXT, BLOB or no type -> BLOB,
    REAL/FLOA/DOUB -> REAL, anything else -> NUMERIC."""
    import corrosion_amd._lib as L
    f = L.lib().corro_affinity_of_type
    cases = {b"INTEGER": 3, b"int": 3, b"BIGINT": 3, b"TEXT": 1, b"VARCHAR(10)": 1, b"CLOB": 1, b"BLOB": 0,
             b"": 0, b"REAL": 4, b"DOUBLE PRECISION": 4, b"FLOAT": 4, b"NUMERIC": 2, b"BOOLEAN": 2,
             b"DECIMAL(10,5)": 2, b"FLOATING POINT": 3, b"CHARINT": 3}
    for t, a in cases.items():
        assert f(t) == a, t
