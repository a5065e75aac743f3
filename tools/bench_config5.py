"""Timing probe for BASELINE.json configs[4] (adversarial mix: 8 tables, Zipf(1.1) hot pks, 30 %
sentinel deletes/resurrects, mixed value classes) through the general merge path.
Not the headline bench (bench.py measures configs[1]); prints one line per size."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1000000,4000000")
    ap.add_argument("--impact", action="store_true")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--pmc", action="store_true",
                    help="HBM traffic per apply from rocprofv3 FETCH_SIZE / WRITE_SIZE passes over a child run "
                         "(first size only; before this process touches the GPU)")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()
    traffic = None
    if args.pmc and not args.pmc_child:
        import bench
        n0 = int(args.sizes.split(",")[0])
        child = [os.path.abspath(__file__), "--pmc-child", "--sizes", str(n0), "--reps", str(args.reps)]
        if args.impact:
            child.append("--impact")
        tb, note, per = bench.pmc_traffic_live(n0, applies=args.reps + 1, timeout=400, child_cmd=child)
        traffic = {"bytes": tb, "source": note, "by_kernel": per}
    import numpy as np
    import torch
    import synth
    import corrosion_amd as ca
    seed = synth.config_seed(5)
    sites = synth.site_ids(1000, seed)
    for n in [int(x) for x in args.sizes.split(",")]:
        t0 = time.perf_counter()
        b = synth.adversarial_batch(n, 1000, 8, 1 << 20, seed)
        gen = time.perf_counter() - t0
        dev = {k: torch.from_numpy(v.view(np.int64) if v.dtype == np.uint64 else
                                   (v.view(np.int32) if v.dtype == np.uint32 else v)).cuda() for k, v in b.items()}
        eng = ca.MergeEngine(synth.adversarial_schema(8), capacity_hint=n, device=0)
        eng.register_sites(sites)
        eng.set_profiling(True)
        times, stages = [], []
        for rep in range(args.reps + 1):
            eng.reset()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            eng.apply(dev, impact=args.impact)
            torch.cuda.synchronize()
            if rep:  # the first apply warms up
                times.append(time.perf_counter() - t0)
                stages.append(eng.last_timings())
        k = int(np.argsort(times)[len(times) // 2])  # the median apply
        dt = times[k]
        print(f"n={n} gen={gen:.1f}s apply={dt*1e3:.2f} ms (median of {args.reps}) rows={eng.count()} "
              f"({n/dt/1e6:.1f} M changes/s) stages={ {s: round(v, 3) for s, v in stages[k].items()} }",
              flush=True)
        # config 5 prices 56 B per change and per output cell (16-B value keys)
        cells = eng.count()
        pipe = sum(stages[k].values())
        alg = 56 * (n + cells)
        print(json.dumps({"metric": "merged column-changes/s (config 5: adversarial)", "value": n / dt,
                          "unit": "merged column-changes/s", "n_gpus": 1, "ms_per_apply": dt * 1e3,
                          "impact": bool(args.impact), "dtype": "int64/16-B blob keys",
                          "config": {"workload": "config 5", "changes": n, "cells": cells, "tables": 8,
                                     "sentinel_frac": 0.3, "zipf": 1.1},
                          "roofline": {"bound": "hbm", "kernel": "apply pipeline (sum of stages)",
                                       "achieved": alg / (pipe * 1e-3) / 1e9, "peak": 8000.0, "unit": "GB/s",
                                       "frac": alg / (pipe * 1e-3) / 1e9 / 8000.0, "alg_bytes": alg,
                                       "pipeline_ms": pipe, "stages_ms": stages[k],
                                       "traffic": traffic["bytes"] if traffic else None,
                                       "traffic_ratio": (traffic["bytes"] / alg) if traffic and traffic["bytes"] else None,
                                       "traffic_source": traffic["source"] if traffic else None,
                                       "traffic_by_kernel": traffic["by_kernel"] if traffic else None}}), flush=True)
        traffic = None  # (measured for the first size only)
        eng.close()


if __name__ == "__main__":
    main()
