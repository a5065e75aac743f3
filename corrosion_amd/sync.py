"""SyncStateV1 / SyncNeedV1 mirror and the batched need diff on the GPU.

Mirrors /root/reference/crates/corro-types/src/sync.rs:
  SyncStateV1 (:79-87), need_len (:90-109), need_len_for_actor (:111-125),
  compute_available_needs (:127-249), SyncNeedV1 (:252-264).
The arithmetic runs in the HIP kernel `k_needs` (csrc/sync_needs.hip) through corro_compute_needs;
this module only flattens HashMaps into CSR entries and rebuilds the HashMap result.
"""
import ctypes as C
from dataclasses import dataclass, field

import numpy as np

from . import _lib as L


@dataclass(frozen=True)
class Full:
    """SyncNeedV1::Full { versions: start..=end }"""
    start: int
    end: int

    def count(self):
        return self.end - self.start + 1


@dataclass(frozen=True)
class Partial:
    """SyncNeedV1::Partial { version, seqs }"""
    version: int
    seqs: tuple

    def count(self):
        return 1


@dataclass
class SyncStateV1:
    actor_id: bytes = b"\0" * 16
    heads: dict = field(default_factory=dict)          # actor -> head
    need: dict = field(default_factory=dict)           # actor -> [(start, end), ...]
    partial_need: dict = field(default_factory=dict)   # actor -> {version: [(s, e), ...]}
    last_cleared_ts: int = None

    def need_len(self):
        full = sum(e - s + 1 for v in self.need.values() for s, e in v)
        part = sum(e - s + 1 for p in self.partial_need.values() for rs in p.values() for s, e in rs)
        return full + part // 50  # sync.rs:106 quirk

    def need_len_for_actor(self, actor):
        return sum(e - s + 1 for s, e in self.need.get(actor, [])) + len(self.partial_need.get(actor, {}))

    def compute_available_needs(self, other, engine):
        """HashMap<ActorId, Vec<SyncNeedV1>>; partials in ascending version order."""
        return batch_compute_available_needs(engine, [(self, other)])[0]


def entries_from_states(pairs):
    """Flatten (ours, theirs) SyncStateV1 pairs into CSR entries. Returns (entries, index) with
    index[e] = (pair number, actor)."""
    E = {k: [] for k in ("their_head", "our_head", "tn_start", "tn_end", "tp_ver", "tps_start",
                         "tps_end", "on_start", "on_end", "op_ver", "ops_start", "ops_end")}
    offs = {k: [0] for k in ("tn_off", "tp_off", "tps_off", "on_off", "op_off", "ops_off")}
    index = []
    for p, (ours, theirs) in enumerate(pairs):
        for actor, head in theirs.heads.items():
            if actor == ours.actor_id or head == 0:  # sync.rs:133-140
                continue
            index.append((p, actor))
            E["their_head"].append(head)
            E["our_head"].append(ours.heads.get(actor, -1))
            for s, e in theirs.need.get(actor, []):
                E["tn_start"].append(s)
                E["tn_end"].append(e)
            offs["tn_off"].append(len(E["tn_start"]))
            tp = theirs.partial_need.get(actor, {})
            for v in sorted(tp):
                E["tp_ver"].append(v)
                for s, e in tp[v]:
                    E["tps_start"].append(s)
                    E["tps_end"].append(e)
                offs["tps_off"].append(len(E["tps_start"]))
            offs["tp_off"].append(len(E["tp_ver"]))
            for s, e in ours.need.get(actor, []):
                E["on_start"].append(s)
                E["on_end"].append(e)
            offs["on_off"].append(len(E["on_start"]))
            op = ours.partial_need.get(actor, {})
            for v in sorted(op):
                E["op_ver"].append(v)
                for s, e in op[v]:
                    E["ops_start"].append(s)
                    E["ops_end"].append(e)
                offs["ops_off"].append(len(E["ops_start"]))
            offs["op_off"].append(len(E["op_ver"]))
    out = {k: np.array(v, dtype=np.int64 if k == "our_head" else np.uint64) for k, v in E.items()}
    for k, v in offs.items():
        out[k] = np.array(v, dtype=np.uint64)
    return out, index


def _needs_host(engine, ent):
    """Run corro_compute_needs on host CSR arrays (two passes). Returns the CSR result dict."""
    lib = L.lib()
    n = len(ent["their_head"])
    keep = []
    s = L.SyncEntries()
    s.n = n
    for k, _ in L.SyncEntries._fields_[1:]:
        a = np.ascontiguousarray(ent[k], dtype=np.int64 if k == "our_head" else np.uint64)
        keep.append(a)
        setattr(s, k, a.ctypes.data if a.size else None)
    o = L.NeedsOut()
    nc = np.zeros(max(n, 1), np.uint64)
    sc = np.zeros(max(n, 1), np.uint64)
    o.need_count, o.seq_count = nc.ctypes.data, sc.ctypes.data
    if n:
        L.check(lib.corro_compute_needs(engine._h, C.byref(s), L.CORRO_MEM_HOST, C.byref(o), 0))
    need_off = np.zeros(n + 1, np.uint64)
    seq_off = np.zeros(n + 1, np.uint64)
    need_off[1:] = np.cumsum(nc[:n])
    seq_off[1:] = np.cumsum(sc[:n])
    T, Ts = int(need_off[-1]), int(seq_off[-1])
    res = {"need_off": need_off, "seq_off": seq_off, "kind": np.zeros(max(T, 1), np.uint8),
           "start": np.zeros(max(T, 1), np.uint64), "end": np.zeros(max(T, 1), np.uint64),
           "sr_off": np.zeros(max(T, 1), np.uint64), "sr_n": np.zeros(max(T, 1), np.uint64),
           "s_start": np.zeros(max(Ts, 1), np.uint64), "s_end": np.zeros(max(Ts, 1), np.uint64)}
    for k in ("need_off", "seq_off", "kind", "start", "end", "sr_off", "sr_n", "s_start", "s_end"):
        setattr(o, k, res[k].ctypes.data)
    if n:
        L.check(lib.corro_compute_needs(engine._h, C.byref(s), L.CORRO_MEM_HOST, C.byref(o), 1))
    for k in ("kind", "start", "end", "sr_off", "sr_n"):
        res[k] = res[k][:T]
    for k in ("s_start", "s_end"):
        res[k] = res[k][:Ts]
    return res


def _needs_device(engine, ent):
    """corro_compute_needs on device-resident CSR entries (dict of CUDA int64 tensors).
    Returns the CSR result as CUDA tensors (two passes, offsets scanned on the device)."""
    import torch
    lib = L.lib()
    n = int(ent["their_head"].shape[0])
    dev = ent["their_head"].device
    s = L.SyncEntries()
    s.n = n
    for k, _ in L.SyncEntries._fields_[1:]:
        a = ent[k]
        setattr(s, k, a.data_ptr() if a.numel() else None)
    nc = torch.empty(max(n, 1), dtype=torch.int64, device=dev)  # pass 0 writes every entry
    sc = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
    o = L.NeedsOut()
    o.need_count, o.seq_count = nc.data_ptr(), sc.data_ptr()
    torch.cuda.current_stream().synchronize()
    L.check(lib.corro_compute_needs(engine._h, C.byref(s), L.CORRO_MEM_DEVICE, C.byref(o), 0))
    need_off = torch.empty(n + 1, dtype=torch.int64, device=dev)
    seq_off = torch.empty(n + 1, dtype=torch.int64, device=dev)
    L.check(lib.corro_scan_offsets(engine._h, nc.data_ptr(), need_off.data_ptr(), n))
    L.check(lib.corro_scan_offsets(engine._h, sc.data_ptr(), seq_off.data_ptr(), n))
    T, Ts = int(need_off[-1].item()), int(seq_off[-1].item())
    # pass 1 writes every output element: no fill needed
    res = {"need_off": need_off, "seq_off": seq_off,
           "kind": torch.empty(max(T, 1), dtype=torch.uint8, device=dev)}
    for k in ("start", "end", "sr_off", "sr_n"):
        res[k] = torch.empty(max(T, 1), dtype=torch.int64, device=dev)
    for k in ("s_start", "s_end"):
        res[k] = torch.empty(max(Ts, 1), dtype=torch.int64, device=dev)
    for k in ("need_off", "seq_off", "kind", "start", "end", "sr_off", "sr_n", "s_start", "s_end"):
        setattr(o, k, res[k].data_ptr())
    torch.cuda.current_stream().synchronize()
    L.check(lib.corro_compute_needs(engine._h, C.byref(s), L.CORRO_MEM_DEVICE, C.byref(o), 1))
    for k in ("kind", "start", "end", "sr_off", "sr_n"):
        res[k] = res[k][:T]
    for k in ("s_start", "s_end"):
        res[k] = res[k][:Ts]
    return res


def _needs_device_1pass(engine, ent):
    """corro_compute_needs_onepass on device-resident CSR entries: one kernel, every input read once
    (outputs sized by corro_needs_bound; re-run at the exact totals in the never-expected case of
    overlapping need ranges exceeding it). Returns the same CSR dict as _needs_device."""
    import torch
    lib = L.lib()
    n = int(ent["their_head"].shape[0])
    dev = ent["their_head"].device
    s = L.SyncEntries()
    s.n = n
    for k, _ in L.SyncEntries._fields_[1:]:
        a = ent[k]
        setattr(s, k, a.data_ptr() if a.numel() else None)
    torch.cuda.current_stream().synchronize()
    ncap, scap = C.c_uint64(), C.c_uint64()
    L.check(lib.corro_needs_bound(engine._h, C.byref(s), L.CORRO_MEM_DEVICE, C.byref(ncap), C.byref(scap)))
    caps = [ncap.value, scap.value]
    while True:
        res = {"need_off": torch.empty(n + 1, dtype=torch.int64, device=dev),
               "seq_off": torch.empty(n + 1, dtype=torch.int64, device=dev),
               "kind": torch.empty(max(caps[0], 1), dtype=torch.uint8, device=dev)}
        for k in ("start", "end", "sr_off", "sr_n"):
            res[k] = torch.empty(max(caps[0], 1), dtype=torch.int64, device=dev)
        for k in ("s_start", "s_end"):
            res[k] = torch.empty(max(caps[1], 1), dtype=torch.int64, device=dev)
        o = L.NeedsOut()
        for k in ("need_off", "seq_off", "kind", "start", "end", "sr_off", "sr_n", "s_start", "s_end"):
            setattr(o, k, res[k].data_ptr())
        tot = (C.c_uint64 * 2)()
        rc = lib.corro_compute_needs_onepass(engine._h, C.byref(s), C.byref(o), caps[0], caps[1], tot)
        if rc == -6 and (tot[0] > caps[0] or tot[1] > caps[1]):
            caps = [tot[0], tot[1]]
            continue
        L.check(rc)
        break
    if n == 0:
        res["need_off"].zero_()
        res["seq_off"].zero_()
    T, Ts = tot[0], tot[1]
    for k in ("kind", "start", "end", "sr_off", "sr_n"):
        res[k] = res[k][:T]
    for k in ("s_start", "s_end"):
        res[k] = res[k][:Ts]
    return res


def _needs_device_packed(engine, ent):
    """corro_compute_needs_packed on device-resident CSR entries: one kernel, no count pass; outputs
    in the workgroup-padded packed layout (slots sized by corro_needs_bound). Returns CUDA tensors
    need_off, need_count, range (2 per slot), kind, s_start, s_end."""
    import torch
    lib = L.lib()
    n = int(ent["their_head"].shape[0])
    dev = ent["their_head"].device
    s = L.SyncEntries()
    s.n = n
    for k, _ in L.SyncEntries._fields_[1:]:
        a = ent[k]
        setattr(s, k, a.data_ptr() if a.numel() else None)
    torch.cuda.current_stream().synchronize()
    ncap, scap = C.c_uint64(), C.c_uint64()
    L.check(lib.corro_needs_bound(engine._h, C.byref(s), L.CORRO_MEM_DEVICE, C.byref(ncap), C.byref(scap)))
    res = {"need_off": torch.empty(max(n, 1), dtype=torch.int64, device=dev),
           "need_count": torch.empty(max(n, 1), dtype=torch.int32, device=dev),
           "range": torch.empty(2 * max(ncap.value, 1), dtype=torch.int64, device=dev),
           "kind": torch.empty(max(ncap.value, 1), dtype=torch.uint8, device=dev),
           "s_start": torch.empty(max(scap.value, 1), dtype=torch.int64, device=dev),
           "s_end": torch.empty(max(scap.value, 1), dtype=torch.int64, device=dev)}
    o = L.NeedsPackedOut()
    for k in ("need_off", "need_count", "range", "kind", "s_start", "s_end"):
        setattr(o, k, res[k].data_ptr())
    L.check(lib.corro_compute_needs_packed(engine._h, C.byref(s), C.byref(o), ncap.value, scap.value))
    res["need_off"], res["need_count"] = res["need_off"][:n], res["need_count"][:n]
    return res


def packed_to_csr(res):
    """The packed layout as the CSR dict of corro_compute_needs (numpy, host): need_off / seq_off
    (n+1), kind, start, end, sr_off, sr_n, s_start, s_end."""
    import numpy as np
    g = {k: (v.cpu().numpy() if hasattr(v, "cpu") else np.asarray(v)) for k, v in res.items()}
    cnt = g["need_count"].astype(np.int64)
    n = len(cnt)
    need_off = np.zeros(n + 1, np.int64)
    need_off[1:] = np.cumsum(cnt)
    T = int(need_off[-1])
    slot = np.repeat(g["need_off"].astype(np.int64) - need_off[:-1], cnt) + np.arange(T)
    rng = g["range"].view(np.uint64).reshape(-1, 2)[slot]
    kind = g["kind"][slot]
    part = kind == 1
    first = (rng[:, 1] >> np.uint64(24)).astype(np.int64)
    sr_n = np.where(part, (rng[:, 1] & np.uint64(0xFFFFFF)).astype(np.int64), 0)
    ent_of = np.repeat(np.arange(n), cnt)
    seq_cnt = np.bincount(ent_of, weights=sr_n, minlength=n).astype(np.int64) if T else np.zeros(n, np.int64)
    seq_off = np.zeros(n + 1, np.int64)
    seq_off[1:] = np.cumsum(seq_cnt)
    # seq ranges of the partials in need order, compacted
    sr_off = np.zeros(T, np.int64)
    sr_off[1:] = np.cumsum(sr_n)[:-1]
    src = np.repeat(np.where(part, first, 0), sr_n) + (np.arange(int(sr_n.sum())) - np.repeat(sr_off, sr_n))
    full_sr = np.zeros(T, np.int64)  # a Full need's sr_off: the seq ranges emitted before it
    full_sr[:] = sr_off
    return {"need_off": need_off, "seq_off": seq_off, "kind": kind,
            "start": rng[:, 0].astype(np.int64),
            "end": np.where(part, rng[:, 0], rng[:, 1]).astype(np.int64),
            "sr_off": full_sr, "sr_n": sr_n,
            "s_start": g["s_start"][src].astype(np.int64), "s_end": g["s_end"][src].astype(np.int64)}


def decode(res, index, npairs):
    out = [dict() for _ in range(npairs)]
    for e, (p, actor) in enumerate(index):
        lst = []
        for k in range(int(res["need_off"][e]), int(res["need_off"][e + 1])):
            if int(res["kind"][k]) == 0:
                lst.append(Full(int(res["start"][k]), int(res["end"][k])))
            else:
                o, m = int(res["sr_off"][k]), int(res["sr_n"][k])
                lst.append(Partial(int(res["start"][k]),
                                   tuple((int(res["s_start"][j]), int(res["s_end"][j])) for j in range(o, o + m))))
        if lst:
            out[p][actor] = lst
    return out


def batch_compute_available_needs(engine, pairs):
    """compute_available_needs for many (ours, theirs) pairs in one kernel launch pair."""
    ent, index = entries_from_states(pairs)
    res = _needs_host(engine, ent)
    return decode(res, index, len(pairs))
