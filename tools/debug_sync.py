"""Debug probe: config-4 need diff at full size, GPU vs oracle; prints the entries whose outputs
differ (their inputs and both outputs) and saves them as a small JSON case file."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import synth  # noqa: E402
from oracle import oracle as O  # noqa: E402


def entry_inputs(h, e):
    def seg(off, *arrs):
        a, b = int(h[off][e]), int(h[off][e + 1])
        return [[int(x[i]) for x in arrs] for i in range(a, b)], (a, b)
    tn, _ = seg("tn_off", h["tn_start"], h["tn_end"])
    on, _ = seg("on_off", h["on_start"], h["on_end"])
    tp = []
    for k in range(int(h["tp_off"][e]), int(h["tp_off"][e + 1])):
        tp.append([int(h["tp_ver"][k]), [[int(h["tps_start"][j]), int(h["tps_end"][j])]
                                         for j in range(int(h["tps_off"][k]), int(h["tps_off"][k + 1]))]])
    op = []
    for k in range(int(h["op_off"][e]), int(h["op_off"][e + 1])):
        op.append([int(h["op_ver"][k]), [[int(h["ops_start"][j]), int(h["ops_end"][j])]
                                         for j in range(int(h["ops_off"][k]), int(h["ops_off"][k + 1]))]])
    return {"their_head": int(h["their_head"][e]), "our_head": int(h["our_head"][e]), "their_need": tn,
            "our_need": on, "their_partials": tp, "our_partials": op}


def outputs(r, e):
    a, b = int(r["need_off"][e]), int(r["need_off"][e + 1])
    out = []
    for q in range(a, b):
        s0, n = int(r["sr_off"][q]), int(r["sr_n"][q])
        out.append([int(r["kind"][q]), int(r["start"][q]), int(r["end"][q]),
                    [[int(r["s_start"][j]), int(r["s_end"][j])] for j in range(s0, s0 + n)]])
    return out


def main():
    import torch
    import corrosion_amd as ca
    from corrosion_amd.sync import _needs_device
    npairs = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    ent = synth.sync_entries_torch(npairs, 64, synth.config_seed(4), device="cuda")
    e = ca.MergeEngine({"t": ["a"]}, capacity_hint=1024)
    got = {k: (v.cpu().numpy().view(np.uint64) if v.dtype == torch.int64 else v.cpu().numpy())
           for k, v in _needs_device(e, ent).items()}
    h = {k: v.cpu().numpy() for k, v in ent.items()}
    exp = O.needs_parallel(h, nthreads=16)
    cg, ce = np.diff(got["need_off"].astype(np.int64)), np.diff(exp["need_off"].astype(np.int64))
    sg, se = np.diff(got["seq_off"].astype(np.int64)), np.diff(exp["seq_off"].astype(np.int64))
    bad = np.nonzero((cg != ce) | (sg != se))[0]
    print(f"entries {len(cg)}, count mismatches {len(bad)}", flush=True)
    cases = []
    for i in bad[:8]:
        i = int(i)
        inp = entry_inputs(h, i)
        print(json.dumps({"entry": i, "in": inp, "gpu": outputs(got, i), "oracle": outputs(exp, i)}), flush=True)
        cases.append({"in": inp, "oracle": outputs(exp, i), "gpu": outputs(got, i)})
    os.makedirs("gpurun_out/dbg", exist_ok=True)
    json.dump(cases, open("gpurun_out/dbg/sync_cases.json", "w"))


if __name__ == "__main__":
    main()
