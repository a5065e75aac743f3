"""SyncStateV1-shaped test data <-> CSR entries (shared by oracle and GPU tests)."""
import numpy as np


def entries_from_pairs(pairs):
    """pairs: list of (our, their) per (pair, actor) entry; each side is
    {"head": int|None, "need": [[s,e],...], "partials": {ver: [[s,e],...]}}.
    Partials are iterated in ascending version order (canonical form of the HashMap order)."""
    E = {k: [] for k in ("their_head", "our_head", "tn_start", "tn_end", "tp_ver", "tps_start",
                         "tps_end", "on_start", "on_end", "op_ver", "ops_start", "ops_end")}
    tn_off, tp_off, tps_off, on_off, op_off, ops_off = [0], [0], [0], [0], [0], [0]
    for our, their in pairs:
        E["their_head"].append(their["head"])
        E["our_head"].append(-1 if our.get("head") is None else our["head"])
        for s, e in their.get("need", []):
            E["tn_start"].append(s); E["tn_end"].append(e)
        tn_off.append(len(E["tn_start"]))
        for v in sorted(their.get("partials", {}), key=int):
            E["tp_ver"].append(int(v))
            for s, e in their["partials"][v]:
                E["tps_start"].append(s); E["tps_end"].append(e)
            tps_off.append(len(E["tps_start"]))
        tp_off.append(len(E["tp_ver"]))
        for s, e in our.get("need", []):
            E["on_start"].append(s); E["on_end"].append(e)
        on_off.append(len(E["on_start"]))
        for v in sorted(our.get("partials", {}), key=int):
            E["op_ver"].append(int(v))
            for s, e in our["partials"][v]:
                E["ops_start"].append(s); E["ops_end"].append(e)
            ops_off.append(len(E["ops_start"]))
        op_off.append(len(E["op_ver"]))
    out = {k: np.array(v, dtype=np.int64 if k == "our_head" else np.uint64) for k, v in E.items()}
    for k, v in (("tn_off", tn_off), ("tp_off", tp_off), ("tps_off", tps_off), ("on_off", on_off),
                 ("op_off", op_off), ("ops_off", ops_off)):
        out[k] = np.array(v, dtype=np.uint64)
    return out


def decode_needs(res, n):
    """CSR result -> list (per entry) of ('full', s, e) / ('partial', v, [(s,e),...])"""
    out = []
    for e in range(n):
        lst = []
        for k in range(int(res["need_off"][e]), int(res["need_off"][e + 1])):
            if int(res["kind"][k]) == 0:
                lst.append(("full", int(res["start"][k]), int(res["end"][k])))
            else:
                o, m = int(res["sr_off"][k]), int(res["sr_n"][k])
                lst.append(("partial", int(res["start"][k]),
                            [(int(res["s_start"][j]), int(res["s_end"][j])) for j in range(o, o + m)]))
        out.append(lst)
    return out


def kat_expect(expect):
    out = []
    for x in expect:
        if x[0] == "full":
            out.append(("full", x[1], x[2]))
        else:
            out.append(("partial", x[1], [tuple(r) for r in x[2]]))
    return out


def pairs_from_cases(cases):
    """tests/golden/sync_inverted_cases.json entries -> (our, their) pairs for entries_from_pairs."""
    pairs = []
    for c in cases:
        x = c["in"]
        our = {"head": None if x["our_head"] < 0 else x["our_head"], "need": x["our_need"],
               "partials": {str(v): r for v, r in x["our_partials"]}}
        their = {"head": x["their_head"], "need": x["their_need"],
                 "partials": {str(v): r for v, r in x["their_partials"]}}
        pairs.append((our, their))
    return pairs


def expected_from_cases(cases):
    out = []
    for c in cases:
        lst = []
        for kind, s, e, seqs in c["oracle"]:
            lst.append(("full", s, e) if kind == 0 else ("partial", s, [tuple(r) for r in seqs]))
        out.append(lst)
    return out
