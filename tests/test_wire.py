"""Host side of the wire format (corrosion_amd/wire.py) on CPU: speedy layout facts of the
changeset types and the pack_columns / unpack_columns pk encoding (pubsub.rs:2304-2451)."""
import struct

import pytest

from corrosion_amd import wire
from corrosion_amd.agent import Change, ChangeV1, Empty, EmptySet, Full

A = bytes(range(16))


def test_change_layout():
    ch = Change("t", 5, "a", "hi", 3, 7, 2, A, 1)
    b = wire.encode_change(ch)
    # "t": u32 1 + 't'; pk: u32 3 + [1, 0x09, 5]; "a"; Text tag 3 + u32 2 + "hi"; cv i64; dbv u64; seq u64; site; cl
    exp = (struct.pack("<I", 1) + b"t" + struct.pack("<I", 3) + bytes([1, 0x09, 5]) + struct.pack("<I", 1) + b"a" +
           b"\x03" + struct.pack("<I", 2) + b"hi" + struct.pack("<qQQ", 3, 7, 2) + A + struct.pack("<q", 1))
    assert b == exp


def test_changeset_variants_and_messages():
    full = ChangeV1(A, Full(9, [], (0, 3), 3, ts=77))
    assert wire.encode_changev1(full) == A + struct.pack("<IQI", 1, 9, 0) + struct.pack("<QQQQ", 0, 3, 3, 77)
    emp = ChangeV1(A, Empty((4, 6), ts=None))
    assert wire.encode_changev1(emp) == A + struct.pack("<IQQ", 0, 4, 6) + b"\x00"
    es = ChangeV1(A, EmptySet([(1, 2), (5, 5)], ts=8))
    assert wire.encode_changev1(es) == A + struct.pack("<II", 2, 2) + struct.pack("<QQQQQ", 1, 2, 5, 5, 8)
    m = wire.encode_sync_changeset(emp)
    assert m[:8] == struct.pack("<II", 0, 1)
    u = wire.encode_uni_change(emp, cluster_id=3)
    assert u[:12] == struct.pack("<III", 0, 0, 0) and u[-2:] == struct.pack("<H", 3)
    f = wire.frame(b"abc")
    assert f == b"\x00\x00\x00\x03abc"


@pytest.mark.parametrize("v,packed", [(0, [1, 1]), (5, [1, 0x09, 5]), (300, [1, 0x11, 1, 44]),
                                      (-1, [1, 0x41] + [0xFF] * 8), (1 << 40, [1, 0x31, 1, 0, 0, 0, 0, 0])])
def test_pack_int_pk(v, packed):
    assert list(wire.pack_int_pk(v)) == packed


def test_unpack_sign_extends_like_get_int():
    # 200 packs into one byte (0xC8); bytes::Buf::get_int(1) sign-extends it back to -56
    assert wire.unpack_int_pk(wire.pack_int_pk(200)) == -56
    for v in (0, 1, 127, 300, -1, -129, 1 << 40, -(1 << 62)):
        if v < 0 or wire.pack_int_pk(v)[2:3] < b"\x80":
            assert wire.unpack_int_pk(wire.pack_int_pk(v)) == v
