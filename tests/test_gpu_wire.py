"""GPU wire decode (corro_decode_frames, csrc/wire.hip) against the host restatement of the speedy
layout (corrosion_amd/wire.py): frames encoded on the host, decoded on the GPU, compared field
by field with what the engine's own host-side encoding of the same objects gives; then bytes ->
merge end to end (Agent.process_frames) against the same objects applied directly. Parity is
against the restated speedy 0.8.7 layout: the reference holds no encoded fixtures."""
import numpy as np
import pytest

from corrosion_amd import wire
from corrosion_amd.agent import Change, ChangeV1, Empty, EmptySet, Full, encode_value

pytestmark = pytest.mark.gpu

SCHEMA = {"users": ["name", "age", "blob"], "t2": ["x"]}
ACT = [bytes([i] * 16) for i in range(1, 6)]


def rand_changes(rng, n, actor, version):
    out = []
    for k in range(n):
        t = "users" if rng.random() < 0.8 else ("t2" if rng.random() < 0.9 else "nope")
        cols = SCHEMA.get(t, ["zz"])
        cid = "-1" if rng.random() < 0.1 else (cols[int(rng.integers(len(cols)))] if rng.random() < 0.95 else "bad")
        r = rng.random()
        if cid == "-1":
            val = None
        elif r < 0.4:
            val = int(rng.integers(-(1 << 62), 1 << 62))
        elif r < 0.55:
            val = float(rng.choice([0.0, -2.5, 1e300, 3.25]))
        elif r < 0.75:
            val = "".join(chr(97 + int(x)) for x in rng.integers(0, 26, int(rng.integers(0, 41))))
        elif r < 0.9:  # (values past 16 bytes travel as val_off / val_size into the frame bytes)
            val = bytes(rng.integers(0, 256, int(rng.integers(0, 41))).astype(np.uint8))
        else:
            val = None
        pk = int(rng.choice([int(rng.integers(0, 128)), int(rng.integers(-(1 << 40), 1 << 40)), 1 << 60]))
        site = ACT[int(rng.integers(len(ACT)))] if rng.random() < 0.3 else actor
        out.append(Change(t, pk, cid, val, int(rng.integers(1, 9)), version, k, site, int(rng.choice([1, 1, 1, 2, 3]))))
    return out


def expected_fields(eng, ch, ts):
    try:
        tc = eng.lookup(ch.table, ch.cid)
    except Exception:
        tc = 0xFFFFFFFF
    vt, v0, v1, ln = encode_value(ch.val)
    pk = wire.unpack_int_pk(wire.pack_int_pk(ch.pk)) & 0xFFFFFFFFFFFFFFFF
    site = int(eng.register_sites(np.frombuffer(ch.site_id, np.uint8).reshape(1, 16))[0])
    return (pk, tc, ch.col_version, ch.db_version, ch.cl, ch.seq, site, v0, v1, vt, ln, ts)


def got_fields(dec, i):
    c = dec["changes"]
    return tuple(int(c[k][i]) for k in ("pk", "table_cid", "col_version", "db_version", "cl", "seq", "site", "val0",
                                         "val1", "val_type", "val_len", "ts"))


def got_long(dec, i):
    """the bytes of decoded change i's long value (val_off / val_size into the frame buffer)"""
    c = dec["changes"]
    o, n = int(c["val_off"][i]), int(c["val_size"][i])
    return bytes(c["val_data"][o:o + n])


@pytest.mark.parametrize("payload", [wire.PAYLOAD_SYNC, wire.PAYLOAD_UNI])
def test_decode_roundtrip(payload):
    import corrosion_amd as ca
    rng = np.random.default_rng(3 + payload)
    msgs = []
    for i in range(300):
        a = ACT[i % 4]
        r = rng.random()
        if r < 0.8:
            n = int(rng.integers(0, 60))
            msgs.append(ChangeV1(a, Full(i + 1, rand_changes(rng, n, a, i + 1), (0, max(n - 1, 0)), max(n - 1, 0),
                                         ts=int(rng.integers(0, 1 << 62)))))
        elif r < 0.9:
            msgs.append(ChangeV1(a, Empty((i, i + 3), ts=None if rng.random() < 0.5 else 12345)))
        else:
            msgs.append(ChangeV1(a, EmptySet([(1, 2), (i, i + 9)], ts=99)))
    eng = ca.MergeEngine(SCHEMA, capacity_hint=1 << 14)
    dec = eng.decode_frames(wire.frames(msgs, payload), payload)
    assert dec["nframes"] == len(msgs) and (dec["status"] == 0).all()
    sets = 0
    for i, m in enumerate(msgs):
        cs = dec["cs"][i]
        import ctypes
        assert ctypes.string_at(cs.actor_id, 16) == m.actor_id
        assert cs.site == int(eng.register_sites(np.frombuffer(m.actor_id, np.uint8).reshape(1, 16))[0])
        x = m.changeset
        if isinstance(x, Full):
            assert (cs.kind, cs.version_start, cs.seq_start, cs.seq_end, cs.last_seq, cs.ts) == \
                   (0, x.version, x.seqs[0], x.seqs[1], x.last_seq, x.ts)
            assert cs.change_count == len(x.changes)
            for k, ch in enumerate(x.changes):
                assert got_fields(dec, cs.change_off + k) == expected_fields(eng, ch, x.ts), (i, k)
                if dec["changes"]["val_len"][cs.change_off + k] == 255:
                    raw = ch.val.encode() if isinstance(ch.val, str) else bytes(ch.val)
                    assert got_long(dec, cs.change_off + k) == raw
        elif isinstance(x, Empty):
            assert (cs.kind, cs.version_start, cs.version_end, cs.ts) == (1, x.versions[0], x.versions[1], x.ts or 0)
        else:
            assert cs.kind == 2 and cs.change_count == len(x.versions) and cs.ts == x.ts
            got = [(int(dec["set_start"][cs.change_off + k]), int(dec["set_end"][cs.change_off + k]))
                   for k in range(cs.change_count)]
            assert got == x.versions
            sets += len(x.versions)
    assert len(dec["set_start"]) == sets


def test_decode_large_frames_and_errors():
    """A frame above the 16 KB LDS stage and with more than 1024 changes (global paths), a
    non-changeset sync message, a truncated changeset, a 17-byte TEXT (decoded as a long value)
    and a text pk of a table not marked interned (outside the encoding)."""
    import corrosion_amd as ca
    import struct
    rng = np.random.default_rng(9)
    big = ChangeV1(ACT[0], Full(1, [Change("users", k, "age", k, 1, 1, k, ACT[0], 1) for k in range(1500)],
                                (0, 1499), 1499, ts=5))
    mid = ChangeV1(ACT[1], Full(2, rand_changes(rng, 200, ACT[1], 2), (0, 199), 199, ts=6))
    clock = struct.pack("<IIQ", 0, 2, 42)          # SyncMessage::V1(SyncMessageV1::Clock(ts))
    good = wire.encode_sync_changeset(mid)
    trunc = wire.encode_sync_changeset(ChangeV1(ACT[2], Full(3, rand_changes(rng, 5, ACT[2], 3), (0, 4), 4, ts=1)))[:-20]
    long_text = wire.encode_sync_changeset(ChangeV1(ACT[3], Full(4, [Change("users", 1, "name", "x" * 17, 1, 4, 0,
                                                                            ACT[3], 1)], (0, 0), 0, ts=1)))
    text_pk = wire.encode_sync_changeset(ChangeV1(ACT[3], Full(5, [Change("users", b"\x01\x03\x01a", "name", "y", 1, 5,
                                                                          0, ACT[3], 1)], (0, 0), 0, ts=1)))
    # a Full changeset that claims 2^32-1 changes in a 25-byte body: malformed, and sizes nothing
    huge = struct.pack("<II", 0, 1) + bytes(ACT[4]) + struct.pack("<IQI", 1, 7, 0xFFFFFFFF)
    buf = b"".join(wire.frame(x) for x in (wire.encode_sync_changeset(big), clock, good, trunc, long_text, text_pk,
                                           huge))
    eng = ca.MergeEngine(SCHEMA, capacity_hint=1 << 14)
    dec = eng.decode_frames(buf)
    assert list(dec["status"]) == [0, 1, 0, -1, 0, -6, -1]
    i = dec["cs"][4].change_off
    assert dec["changes"]["val_len"][i] == 255 and got_long(dec, i) == b"x" * 17
    assert dec["cs"][6].change_count == 0
    assert len(dec["changes"]["pk"]) <= 1500 + 200 + 5 + 1 + 1
    cs0 = dec["cs"][0]
    assert cs0.change_count == 1500 and cs0.last_seq == 1499 and cs0.ts == 5
    for k in (0, 777, 1499):
        assert got_fields(dec, cs0.change_off + k) == expected_fields(eng, big.changeset.changes[k], 5)
    cs2 = dec["cs"][2]
    for k, ch in enumerate(mid.changeset.changes):
        assert got_fields(dec, cs2.change_off + k) == expected_fields(eng, ch, 6)


def test_process_frames_equals_process_objects():
    """bytes -> GPU decode -> process_multiple_changes gives the state that applying the same
    ChangeV1 objects gives (known outcomes, rows, db_versions, gap bookkeeping)."""
    import corrosion_amd as ca
    rng = np.random.default_rng(11)
    msgs = []
    for v in range(1, 120):
        a = ACT[v % 3]
        ch = [c for c in rand_changes(rng, int(rng.integers(1, 30)), a, v) if c.table != "nope" and c.cid != "bad"]
        for k, c in enumerate(ch):
            c.seq = k
            # keep pks that pack_columns / unpack_columns round-trip (a value whose top packed bit
            # is set comes back sign-extended, a different row key on the wire path)
            if wire.unpack_int_pk(wire.pack_int_pk(c.pk)) != c.pk:
                c.pk = -abs(c.pk)
        if not ch:
            msgs.append(ChangeV1(a, Empty((v, v))))
        elif rng.random() < 0.15:                  # partial: first half of the seqs
            h = max(1, len(ch) // 2)
            msgs.append(ChangeV1(a, Full(v, ch[:h], (0, h - 1), len(ch) - 1, ts=v)))
        else:
            msgs.append(ChangeV1(a, Full(v, ch, (0, len(ch) - 1), len(ch) - 1, ts=v)))
    x = ca.agent.Agent(SCHEMA, capacity_hint=1 << 14)
    y = ca.agent.Agent(SCHEMA, capacity_hint=1 << 14)
    for a in ACT:                                   # same site ordinals on both
        x.site(a)
        y.site(a)
    rx = x.process_multiple_changes(msgs)
    ry, st = y.process_frames(wire.frames(msgs))
    assert (st == 0).all() and rx.known == ry.known

    assert canon(x.engine) == canon(y.engine)
    assert list(x.engine.db_versions()) == list(y.engine.db_versions())
    for a in ACT[:3]:
        assert x.bookie.needed(a) == y.bookie.needed(a) and x.bookie.last(a) == y.bookie.last(a)


def canon(e):
    """the state's rows, comparable across engines: long values by their bytes, interned row keys
    by their packed pks"""
    r = e.export()
    longs = r["long_values"]
    keys = ("table_cid", "pk", "val_type", "val0", "val1", "val_len", "col_version", "db_version", "site", "cl",
            "seq", "ts")
    cols = [r[k].tolist() for k in keys]
    for i, b in longs.items():
        cols[4][i] = b
    for t, (name, _c) in enumerate(e.schema):
        if name in e.interned:
            idx = [i for i, tc in enumerate(cols[0]) if tc >> 16 == t]
            for i, pk in zip(idx, e.pk_bytes(t, [cols[1][i] for i in idx])):
                cols[1][i] = pk
    return sorted(zip(*cols), key=repr)


WSCHEMA = {"tests": ["text"], "testsblob": ["text"], "wide": ["int", "float", "blob"]}


def test_process_frames_interned_pks_and_long_values():
    """corro-tests' BLOB-pk and composite-pk tables (corro-tests/src/lib.rs:32-52) over the wire:
    interned pks and long values decoded on the GPU give the state the same objects give."""
    import corrosion_amd as ca
    rng = np.random.default_rng(12)
    from tests.test_gpu_pk import _pack
    msgs = []
    for v in range(1, 80):
        a = ACT[v % 3]
        ch = []
        for k in range(int(rng.integers(1, 25))):
            t = ["tests", "testsblob", "wide"][int(rng.integers(0, 3))]
            j = int(rng.integers(0, 30))
            pk = j if t == "tests" else (_pack([bytes([j]) * (1 + j % 4)]) if t == "testsblob"
                                         else _pack([j.to_bytes(8, "big"), str(j % 5)]))
            cols = WSCHEMA[t]
            cid = cols[int(rng.integers(0, len(cols)))]
            if cid in ("text", "blob"):
                n = int(rng.integers(0, 50))
                val = "t" * n if cid == "text" else bytes([j]) * n
            else:
                val = int(rng.integers(0, 3)) if cid == "int" else 0.5
            ch.append(Change(t, pk, cid, val, int(rng.integers(1, 3)), v, k, a, 1))
        msgs.append(ChangeV1(a, Full(v, ch, (0, len(ch) - 1), len(ch) - 1, ts=v)))
    x = ca.agent.Agent(WSCHEMA, capacity_hint=1 << 12, interned=("testsblob", "wide"))
    y = ca.agent.Agent(WSCHEMA, capacity_hint=1 << 12, interned=("testsblob", "wide"))
    for a in ACT:
        x.site(a)
        y.site(a)
    rx = x.process_multiple_changes(msgs)
    ry, st = y.process_frames(wire.frames(msgs))
    assert (st == 0).all() and rx.known == ry.known
    cx, cy = canon(x.engine), canon(y.engine)
    assert cx == cy
    assert any(isinstance(row[4], bytes) for row in cx)          # long values present
    assert any(isinstance(row[1], bytes) for row in cx)          # interned pks present


def test_decode_corrupt_length_prefixes():
    """A length prefix past the frame end (table, pk, cid or value length, each set to 2^32 - 16)
    marks only that frame malformed; the speculative walk's predictions never hide it, and a
    neighbouring good frame decodes unchanged."""
    import corrosion_amd as ca
    import struct
    rng = np.random.default_rng(21)
    ch = [Change("users", 5 + k, "name", "abcdefgh", 1, 1, k, ACT[0], 1) for k in range(6)]
    good = wire.encode_sync_changeset(ChangeV1(ACT[0], Full(1, ch, (0, 5), 5, ts=3)))
    # change 3's fields: payload offset 40 is change 0; every change here has the same size
    size = (len(good) - 40 - 32) // 6
    base = 40 + 3 * size
    lt = struct.unpack_from("<I", good, base)[0]
    lp = struct.unpack_from("<I", good, base + 4 + lt)[0]
    lc = struct.unpack_from("<I", good, base + 8 + lt + lp)[0]
    offs = [base, base + 4 + lt, base + 8 + lt + lp, base + 12 + lt + lp + lc + 1]  # table, pk, cid, value
    bad = []
    for o in offs:
        b = bytearray(good)
        struct.pack_into("<I", b, o, 0xFFFFFFF0)
        bad.append(bytes(b))
    mixed = wire.encode_sync_changeset(ChangeV1(ACT[1], Full(2, rand_changes(rng, 40, ACT[1], 2), (0, 39), 39, ts=4)))
    buf = b"".join(wire.frame(x) for x in bad + [good, mixed])
    eng = ca.MergeEngine(SCHEMA, capacity_hint=1 << 12)
    dec = eng.decode_frames(buf)
    assert list(dec["status"]) == [-1, -1, -1, -1, 0, 0]
    cs = dec["cs"][4]
    for k, c in enumerate(ch):
        assert got_fields(dec, cs.change_off + k) == expected_fields(eng, c, 3)
