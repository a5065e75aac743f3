"""Full-size parity: the north-star correctness criterion at >= 512M column changes.

Generates BASELINE.json config 3's distribution (2^29 changes, 1 table, 4 INTEGER columns, pk
uniform over 2^25, 1000 actors, cl = 1) in HBM, merges it on one MI355X
through the C ABI (one batch, or --batches K consecutive batches folded into the same state), and
checks the result against the oracle's pk-sharded fold (oracle/crsql_fold.c of_apply_sharded, the
same rules as the sequential restatement, run on the host cores) on the same changes:

  * per-change crsql_rows_impacted() growth: array equality (all 2^29 flags),
  * merged crsql_changes rows: row count + order-independent digests (sum and xor of per-row
    64-bit hashes over every output field, oracle rows_digest vs ShardedFold.digest),
  * crsql_db_versions: array equality.

Test infrastructure: the oracle is the checker here, never the thing measured. Prints one progress
line per step and a final JSON line; exits 1 on any mismatch.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def log(msg):
    print(f"[{time.strftime('%H:%M:%S')}] {msg}", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--changes", type=int, default=1 << 29)
    ap.add_argument("--pk-space", type=int, default=1 << 25)
    ap.add_argument("--batches", type=int, default=1)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--out", default="gpurun_out/parity_scale.json")
    args = ap.parse_args()

    import torch
    import corrosion_amd as ca
    import synth
    from oracle import oracle as O

    n_total, K = args.changes, args.batches
    per = n_total // K
    sites = synth.site_ids(1000, 1)
    eng = ca.MergeEngine({"t": ["a", "b", "c", "d"]}, capacity_hint=n_total, device=0)
    eng.register_sites(sites)
    fold = O.ShardedFold(sites, nshards=64, nthreads=args.threads)
    res = {"changes": n_total, "batches": K, "pk_space": args.pk_space, "impact_mismatches": 0}
    t_gpu = t_cpu = 0.0
    for k in range(K):
        seed = synth.config_seed(3) + k
        b = synth.uniform_batch_torch(per, 1000, args.pk_space, 4, seed=seed, device="cuda")
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        imp = eng.apply(b, impact=True)
        torch.cuda.synchronize()
        t_gpu += time.perf_counter() - t0
        imp = imp.cpu().numpy()
        hb = {key: v.cpu().numpy() for key, v in b.items()}
        hb["table_cid"] = hb["table_cid"].view(np.uint32)
        hb["cl"] = hb["cl"].view(np.uint32)
        hb["seq"] = hb["seq"].view(np.uint32)
        hb["site"] = hb["site"].view(np.uint32)
        hb["val0"] = hb["val0"].view(np.uint64)
        hb["pk"] = hb["pk"].view(np.uint64)
        del b
        torch.cuda.empty_cache()
        log(f"batch {k + 1}/{K}: {per} changes merged on the GPU ({t_gpu:.2f} s so far)")
        t0 = time.perf_counter()
        ref = fold.apply(hb)
        t_cpu += time.perf_counter() - t0
        bad = int(np.count_nonzero(imp != ref))
        res["impact_mismatches"] += bad
        log(f"batch {k + 1}/{K}: oracle sharded fold done ({t_cpu:.2f} s so far), impact mismatches {bad}")
        del hb, imp, ref
    rows = eng.export()
    log(f"exported {len(rows['pk'])} rows from the device state")
    dg = O.rows_digest(rows)
    do = fold.digest()
    del rows
    dv_ok = bool(np.array_equal(eng.db_versions(), fold.db_versions()))
    res.update({"rows_gpu": dg[0], "rows_oracle": do[0], "digest_gpu": [hex(dg[1]), hex(dg[2])],
                "digest_oracle": [hex(do[1]), hex(do[2])], "rows_equal": dg == do, "db_versions_equal": dv_ok,
                "gpu_apply_s": round(t_gpu, 3), "oracle_fold_s": round(t_cpu, 3),
                "oracle_threads": args.threads})
    res["pass"] = bool(dg == do and dv_ok and res["impact_mismatches"] == 0)
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res), flush=True)
    eng.close()
    sys.exit(0 if res["pass"] else 1)


if __name__ == "__main__":
    main()
