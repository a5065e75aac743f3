"""Wire format of the changesets corrosion gossips and syncs (host side, and the test encoder).

Restates the speedy 0.8.7 encoding (`corro-speedy` in Cargo.lock; not vendored in the reference)
of the types on the apply path, as derived for them in the reference:
  * little-endian integers; `Vec<T>` / `String` / `&str` / `[u8]` = u32 length + elements;
    `Option<T>` = u8 0/1 + value; derived enums = u32 variant index + fields in declaration order;
    `RangeInclusive<T>` = start, end; fixed arrays raw;
  * `ChangeV1 { actor_id: ActorId (16 raw bytes, actor.rs:91-104), changeset }` and
    `Changeset::{Empty{versions, ts: Option<Timestamp> (default_on_eof)}, Full{version, changes,
    seqs, last_seq, ts}, EmptySet{versions, ts}}` (broadcast.rs:114-148); `Timestamp` = u64
    (broadcast.rs:384-411); `CrsqlDbVersion`/`CrsqlSeq` = u64 (corro-base-types lib.rs:78-175);
  * `Change { table, pk, cid, val, col_version, db_version, seq, site_id, cl }` (change.rs:19-30)
    with `TableName`/`ColumnName` as str (corro-api-types lib.rs:781-850) and the hand-written
    `SqliteValue` encoding: u8 tag 0 Null | 1 i64 | 2 f64 | 3 u32 len + utf8 | 4 u32 len + bytes
    (lib.rs:615-680);
  * frames: tokio `LengthDelimitedCodec` defaults, u32 big-endian length + payload
    (peer/mod.rs:917-929, sync.rs:366-376);
  * `SyncMessage::V1(SyncMessageV1::Changeset(ChangeV1))` = u32 0, u32 1, ChangeV1 (sync.rs:19-30);
    `UniPayload::V1 { data: UniPayloadV1::Broadcast(BroadcastV1::Change(ChangeV1)), cluster_id }`
    = u32 0, u32 0, u32 0, ChangeV1, u16 cluster id (default_on_eof) (broadcast.rs:41-52, 93-96);
  * primary keys: `pack_columns` (pubsub.rs:2304-2384) / `unpack_columns` (:2396-2451).
The GPU decoder (csrc/wire.hip, corro_decode_frames) reads exactly this layout.
"""
import struct

from .agent import Change, ChangeV1, Empty, EmptySet, Full

PAYLOAD_SYNC, PAYLOAD_UNI = 0, 1


def _u32(x):
    return struct.pack("<I", x)


def _u64(x):
    return struct.pack("<Q", x & 0xFFFFFFFFFFFFFFFF)


def _i64(x):
    return struct.pack("<q", x)


def _bytes(b):
    return _u32(len(b)) + bytes(b)


def _num_bytes_i64(val):
    from .serve import num_bytes_needed_i64
    return num_bytes_needed_i64(val)


def pack_int_pk(v):
    """pack_columns([Integer(v)]): count 1, type byte (nbytes << 3 | 1), low nbytes big-endian."""
    n = _num_bytes_i64(v)
    return bytes([1, (n << 3) | 1]) + (v & ((1 << (8 * n)) - 1)).to_bytes(n, "big") if n else bytes([1, 1])


def unpack_int_pk(b):
    """unpack_columns for one INTEGER column: bytes::Buf::get_int(n) sign-extends n big-endian
    bytes (so pack/unpack round-trips only values whose top packed bit matches their sign)."""
    if len(b) < 2 or b[0] != 1 or (b[1] & 7) != 1:
        raise ValueError("not a single INTEGER packed pk")
    n = b[1] >> 3
    if n == 0:
        return 0
    v = int.from_bytes(b[2:2 + n], "big")
    if v >= 1 << (8 * n - 1):
        v -= 1 << (8 * n)
    return v


def encode_value(v):
    if v is None:
        return b"\x00"
    if isinstance(v, bool) or isinstance(v, int):
        return b"\x01" + _i64(v)
    if isinstance(v, float):
        return b"\x02" + struct.pack("<d", v)
    if isinstance(v, str):
        return b"\x03" + _bytes(v.encode())
    return b"\x04" + _bytes(bytes(v))


def encode_change(ch):
    pk = ch.pk if isinstance(ch.pk, (bytes, bytearray)) else pack_int_pk(ch.pk)
    return (_bytes(ch.table.encode()) + _bytes(pk) + _bytes(ch.cid.encode()) + encode_value(ch.val) +
            _i64(ch.col_version) + _u64(ch.db_version) + _u64(ch.seq) + bytes(ch.site_id) + _i64(ch.cl))


def encode_changeset(cs):
    if isinstance(cs, Empty):
        ts = b"\x00" if cs.ts is None else b"\x01" + _u64(cs.ts)
        return _u32(0) + _u64(cs.versions[0]) + _u64(cs.versions[1]) + ts
    if isinstance(cs, Full):
        return (_u32(1) + _u64(cs.version) + _u32(len(cs.changes)) + b"".join(encode_change(c) for c in cs.changes) +
                _u64(cs.seqs[0]) + _u64(cs.seqs[1]) + _u64(cs.last_seq) + _u64(cs.ts or 0))
    if isinstance(cs, EmptySet):
        return _u32(2) + _u32(len(cs.versions)) + b"".join(_u64(s) + _u64(e) for s, e in cs.versions) + _u64(cs.ts or 0)
    raise TypeError(cs)


def encode_changev1(cv):
    return bytes(cv.actor_id) + encode_changeset(cv.changeset)


def encode_sync_changeset(cv):
    """SyncMessage::V1(SyncMessageV1::Changeset(cv))"""
    return _u32(0) + _u32(1) + encode_changev1(cv)


def encode_uni_change(cv, cluster_id=0):
    """UniPayload::V1 { data: UniPayloadV1::Broadcast(BroadcastV1::Change(cv)), cluster_id }"""
    return _u32(0) + _u32(0) + _u32(0) + encode_changev1(cv) + struct.pack("<H", cluster_id)


def frame(payload):
    """LengthDelimitedCodec frame: u32 big-endian length + payload."""
    return struct.pack(">I", len(payload)) + payload


def frames(changes, kind=PAYLOAD_SYNC):
    enc = encode_sync_changeset if kind == PAYLOAD_SYNC else encode_uni_change
    return b"".join(frame(enc(cv)) for cv in changes)
