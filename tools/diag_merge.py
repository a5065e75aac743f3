"""Timing probe of diagnostic library variants (tools/_variants/libcorro_diag<N>.so, built with
-DCORRO_DIAG=N: parts of the fast body switched off or changed, results NOT valid). Each variant runs
in its own child process (CORRO_HIP_LIB); prints the config-2 apply stage times (empty state)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child():
    sys.path.insert(0, ROOT)
    import torch
    import synth
    import corrosion_amd as ca
    n = 1 << 26
    dev = torch.device("cuda", 0)
    eng = ca.MergeEngine({"t": ["a", "b", "c", "d"]}, capacity_hint=n, device=0)
    eng.register_sites(synth.site_ids(1000, 1))
    batch = synth.uniform_batch_torch(n, 1000, 1 << 22, 4, seed=synth.config_seed(2), device=dev)
    impact = os.environ.get("DIAG_IMPACT") == "1"  # the agent path: per-change impact flags
    prep = eng.prepare(batch, impact=impact) if hasattr(eng, "prepare") else None
    eng.set_profiling(True)
    acc = {}
    for it in range(8):
        eng.reset()
        if prep is not None:
            eng.apply_prepared(prep)
        else:
            eng.apply(batch, impact=impact)
        torch.cuda.synchronize()
        if it >= 3:
            for k, v in eng.last_timings().items():
                acc[k] = acc.get(k, 0.0) + v / 5
    print(os.environ.get("CORRO_HIP_LIB", "default"), {k: round(v, 3) for k, v in acc.items()}, flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "child":
        child()
        sys.exit(0)
    libs = [None] + sys.argv[1:]
    for lib in libs:
        env = dict(os.environ)
        if lib:
            env["CORRO_HIP_LIB"] = os.path.abspath(lib)
        r = subprocess.run([sys.executable, "-u", __file__, "child"], env=env, timeout=240)
        if r.returncode != 0:
            sys.exit(r.returncode)
