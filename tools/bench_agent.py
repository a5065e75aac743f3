"""The agent path alone (bench.py's agent_path and agent_e2e fields) for profiling:
    rocprofv3 --kernel-trace --stats -d gpurun_out/agent -- python tools/bench_agent.py
Prints one JSON line with both fields."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import bench
    import synth
    import corrosion_amd as ca
    n = int(os.environ.get("CORRO_AGENT_CHANGES", bench.N_CHANGES))
    reps = int(os.environ.get("CORRO_AGENT_REPS", "5"))
    dev = torch.device("cuda", 0)
    eng = ca.MergeEngine({"t": ["a", "b", "c", "d"]}, capacity_hint=n, device=0)
    eng.register_sites(synth.site_ids(bench.N_ACTORS, 1))
    batch = synth.uniform_batch_torch(n, bench.N_ACTORS, bench.N_PK, bench.N_COLS, seed=synth.config_seed(2),
                                      device=dev)
    torch.cuda.synchronize()
    eng.set_profiling(True)
    only = os.environ.get("CORRO_AGENT_ONLY")  # "path" / "e2e": one of the two (separate kernel traces)
    path = bench.agent_path(eng, batch, n, reps=reps) if only != "e2e" else {"ms": None}
    e2e = bench.agent_e2e(eng, batch, n, path["ms"], reps=reps) if only not in ("path", "mixed") else None
    mixed = bench.agent_e2e_mixed(eng, batch, n, e2e["ms"] if e2e else None, reps=reps) \
        if only in (None, "mixed") else None
    print(json.dumps({"agent_path": path, "agent_e2e": e2e, "agent_e2e_mixed": mixed}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
