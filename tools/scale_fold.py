"""Config-3-shaped scale timing on one MI355X (the SURVEY §8(d) / VERDICT r1 item 3 bar): a 2^26
batch applied into an empty state, 8 consecutive 2^26 batches folded into one growing state (each
batch timed), and one 2^29 apply, all with impact output, in the config-3 distribution (pk space
2^25, 1000 actors, 4 INTEGER columns, cl = 1). Prints one JSON object; parity of the same runs is
tests/test_gpu_scale.py's job. Usage: python tools/scale_fold.py [--out FILE]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import synth  # noqa: E402
import corrosion_amd as ca  # noqa: E402

PER, PK, ACT, NB = 1 << 26, 1 << 25, 1000, 8


def _apply_ms(eng, b, impact=True):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.apply(b, impact=impact)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    sites = synth.site_ids(ACT, 1)
    seed = synth.config_seed(3)
    out = {"shape": "config 3 distribution: pk space 2^25, 1000 actors, 4 INTEGER cols, cl = 1; impact output on"}
    # (1) one 2^26 batch into an empty state (median of 3, after a warm-up)
    eng = ca.MergeEngine({"t": ["a", "b", "c", "d"]}, capacity_hint=PER, device=0)
    eng.register_sites(sites)
    b = synth.uniform_batch_torch(PER, ACT, PK, 4, seed=seed, device="cuda")
    _apply_ms(eng, b)
    empty = []
    for _ in range(3):
        eng.reset()
        empty.append(_apply_ms(eng, b))
    empty.sort()
    out["empty_state_64M_ms"] = empty[1]
    # (2) the 8 x 2^26 fold into one state (the engine sized for the state it will hold: capacity_hint
    # = expected clock rows + changes per apply, as corro_ctx_create documents)
    eng.close()
    eng = ca.MergeEngine({"t": ["a", "b", "c", "d"]}, capacity_hint=PER * NB, device=0)
    eng.register_sites(sites)
    fold = []
    for k in range(NB):
        bk = b if k == 0 else synth.uniform_batch_torch(PER, ACT, PK, 4, seed=seed + k, device="cuda")
        fold.append(_apply_ms(eng, bk))
        print(f"fold batch {k}: {fold[-1]:.2f} ms, state {eng.count()} clock rows", flush=True)
        del bk
    out["fold_8x64M_ms"] = fold
    out["fold_state_rows"] = eng.count()
    out["fold_max_ratio_vs_empty"] = max(fold) / empty[1]
    eng.close()
    del b
    torch.cuda.empty_cache()
    # (3) one 2^29 apply into an empty state
    eng = ca.MergeEngine({"t": ["a", "b", "c", "d"]}, capacity_hint=PER, device=0)
    eng.register_sites(sites)
    big = synth.uniform_batch_torch(PER * NB, ACT, PK, 4, seed=seed, device="cuda")
    eng.set_profiling(True)
    ms = _apply_ms(eng, big)
    out["single_512M_stages_ms"] = eng.last_timings()
    print(f"512M apply: {ms:.2f} ms, stages {out['single_512M_stages_ms']}", flush=True)
    eng.reset()
    ms2 = _apply_ms(eng, big)
    print(f"512M apply again (warm): {ms2:.2f} ms, stages {eng.last_timings()}", flush=True)
    ms = min(ms, ms2)
    out["single_512M_ms"] = ms
    out["single_512M_ratio_vs_64M"] = ms / empty[1]
    out["single_512M_rows"] = eng.count()
    eng.close()
    line = json.dumps(out)
    print(line, flush=True)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
