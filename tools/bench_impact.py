"""Timing probe: config 2 applied WITH per-change impact flags (the agent path: process_multiple_changes
needs crsql_rows_impacted growth per change), vs without. Not the headline bench."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import synth
    import corrosion_amd as ca
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 26
    eng = ca.MergeEngine({"t": ["a", "b", "c", "d"]}, capacity_hint=n, device=0)
    eng.register_sites(synth.site_ids(1000, 1))
    batch = synth.uniform_batch_torch(n, 1000, 1 << 22, 4, seed=synth.config_seed(2), device=torch.device("cuda", 0))
    eng.set_profiling(True)
    for impact in (False, True, False, True):
        eng.reset()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.apply(batch, impact=impact)
        dt = time.perf_counter() - t0
        print(f"impact={impact} apply {dt*1e3:.2f} ms  stages { {k: round(v, 3) for k, v in eng.last_timings().items()} }",
              flush=True)


if __name__ == "__main__":
    main()
