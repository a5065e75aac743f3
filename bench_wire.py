"""Wire-decode benchmark: length-delimited SyncMessage::Changeset frames
-> changeset headers + SoA batch on MI355X (corro_decode_frames).

Workload: 2^20 column changes in Full changesets of 128 changes each (8192 frames, one table of 4
INTEGER columns, 1000 actors, INTEGER values, positive pks below 2^22), encoded on the host with
corrosion_amd/wire.py (speedy layout). One step = one decode call: the device kernels (header
scan + per-frame walk/decode) are timed with HIP events; the call time includes the H2D copy of
the frame bytes and the D2H copy of the decoded batch. Algorithmic bytes: the frame bytes read +
48 B per decoded change written (SURVEY §8(d) SoA). `roofline.traffic` is the HBM bytes per decode
from two rocprofv3 PMC passes over a child run (--no-pmc skips them). Prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
HBM_PEAK_GBS = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--changes", type=int, default=1 << 20)
    ap.add_argument("--per-frame", type=int, default=128)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--no-pmc", action="store_true", help="skip the live rocprofv3 traffic passes")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()
    PMC_RUNS = 3
    traffic = None
    if not args.pmc_child and not args.no_pmc:
        # HBM bytes per decode from rocprofv3 FETCH_SIZE / WRITE_SIZE passes over a child run of this
        # script doing PMC_RUNS decodes, before this process touches the GPU (bench.py's recipe)
        from bench import pmc_traffic_live
        child = [os.path.abspath(__file__), "--pmc-child", "--changes", str(args.changes), "--per-frame",
                 str(args.per_frame)]
        tb, note, per = pmc_traffic_live(0, applies=PMC_RUNS, child_cmd=child)
        if per:  # the decode kernels only
            per = {k: v for k, v in per.items() if "k_wire" in k}
            tb = sum(v["fetch"] + v["write"] for v in per.values())
        traffic = {"bytes": tb, "source": note, "by_kernel": per}
    import numpy as np
    import corrosion_amd as ca
    import synth
    from corrosion_amd import wire
    from corrosion_amd.agent import Change, ChangeV1, Full

    sites = synth.site_ids(1000, 1)
    b = synth.uniform_batch(args.changes, 1000, 1 << 22, 4, synth.config_seed(2))
    cols = ["a", "b", "c", "d"]
    ids = [bytes(s) for s in sites]
    t0 = time.perf_counter()
    frames, P = [], args.per_frame
    for f in range(0, args.changes, P):
        sl = range(f, min(f + P, args.changes))
        a = ids[int(b["site"][f])]
        chs = [Change("t", int(b["pk"][i]), cols[(int(b["table_cid"][i]) & 0xFFFF) - 1], int(b["val0"][i].view(np.int64)),
                      int(b["col_version"][i]), int(b["db_version"][i]), int(b["seq"][i]), ids[int(b["site"][i])], 1)
               for i in sl]
        frames.append(wire.frame(wire.encode_sync_changeset(ChangeV1(a, Full(int(b["db_version"][f]), chs,
                                                                             (0, len(chs) - 1), len(chs) - 1, ts=f)))))
    buf = b"".join(frames)
    enc_s = time.perf_counter() - t0
    eng = ca.MergeEngine({"t": cols}, capacity_hint=args.changes)
    eng.register_sites(sites)
    if args.pmc_child:  # exactly PMC_RUNS decodes, nothing else on the GPU
        for _ in range(PMC_RUNS):
            eng.decode_frames(buf)
        return
    eng.set_profiling(True)
    for _ in range(args.warmup):
        dec = eng.decode_frames(buf)
    kt, t0 = 0.0, time.perf_counter()
    for _ in range(args.steps):
        dec = eng.decode_frames(buf)
        kt += eng.last_timings(apply_only=False)["k_needs_fill"]
    call = (time.perf_counter() - t0) / args.steps
    kt /= args.steps
    assert (dec["status"] == 0).all() and len(dec["changes"]["pk"]) == args.changes
    # pks as unpack_columns reads them back (get_int sign-extends the packed big-endian bytes)
    pk = b["pk"].astype(np.int64)
    nb = np.where(pk < 256, 1, np.where(pk < 65536, 2, 3))
    top = pk >> (8 * nb - 1)
    exp_pk = np.where(top & 1 == 1, pk - (np.int64(1) << (8 * nb)), pk).view(np.uint64)
    assert np.array_equal(dec["changes"]["pk"], exp_pk) and np.array_equal(dec["changes"]["val0"], b["val0"])
    alg = len(buf) + 48 * args.changes
    line = {"metric": "wire decode: decoded column-changes/s (SyncMessage::Changeset frames)",
            "value": args.changes / (kt * 1e-3), "unit": "changes/s (device kernels)", "n_gpus": 1,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": kt, "higher_is_better": True,
            "dtype": "u8", "data": "synthetic (config-2 distribution, speedy-encoded on the host)",
            "config": {"workload": "2^20 changes in Full changesets of %d changes" % P, "frames": len(frames),
                       "bytes": len(buf)},
            "call_ms_with_copies": call * 1e3, "changes_per_s_with_copies": args.changes / call,
            "host_encode_s": enc_s,
            "roofline": {"bound": "hbm", "kernel": "k_wire_hdr + k_wire_decode", "achieved": alg / (kt * 1e-3) / 1e9,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": alg / (kt * 1e-3) / 1e9 / HBM_PEAK_GBS,
                         "traffic": traffic["bytes"] if traffic else None,
                         "traffic_ratio": (traffic["bytes"] / alg) if traffic and traffic["bytes"] else None,
                         "traffic_by_kernel": traffic["by_kernel"] if traffic else None, "alg_bytes": alg}}
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
