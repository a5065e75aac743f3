"""A/B of environment knobs on the config-2 bench: each setting runs `bench.py` (quick: no CPU
baseline, no PMC passes) in a child process, twice, alternating, and one line per run is printed
with ms_per_step and the agent figures. Settings: AB="CORRO_HIST_U=8 CORRO_HIST_U=16;CORRO_SCAT_U=8"
(settings separated by ';', variables inside a setting by spaces; an empty setting = defaults)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(setting):
    env = dict(os.environ)
    for kv in setting.split():
        k, v = kv.split("=", 1)
        env[k] = v
    cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--steps", "10", "--warmup", "3",
           "--no-cpu-baseline", "--no-pmc"]
    out = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=400)
    if out.returncode != 0:
        print(setting or "(defaults)", "FAILED rc", out.returncode, out.stderr[-2000:], flush=True)
        sys.exit(out.returncode)
    line = [x for x in out.stdout.splitlines() if x.startswith("{")][-1]
    d = json.loads(line)
    ag = d.get("agent_path") or {}
    e2e = d.get("agent_e2e") or {}
    print(json.dumps({"setting": setting or "(defaults)", "ms_per_step": d["ms_per_step"],
                      "agent_path_ms": ag.get("ms"), "agent_e2e_ms": e2e.get("ms")}), flush=True)


def main():
    settings = os.environ.get("AB", ";").split(";")
    for _ in range(2):
        for s in settings:
            run(s.strip())


if __name__ == "__main__":
    main()
