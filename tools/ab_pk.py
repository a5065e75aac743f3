"""A/B of device pk intern variants (diagnostic builds in tools/_variants, CORRO_HIP_LIB): each runs
tools/bench_pk.py in a child process, twice, alternating; one line per run (cold and warm ms)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    libs = sys.argv[1:] or [""]
    for _ in range(2):
        for lib in libs:
            env = dict(os.environ)
            if lib:
                env["CORRO_HIP_LIB"] = os.path.join(ROOT, lib)
            out = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tools", "bench_pk.py")], env=env, cwd=ROOT,
                                 capture_output=True, text=True, timeout=300)
            reps = [ln.split(":")[1].split("ms")[0].strip() for ln in out.stdout.splitlines() if ln.startswith("rep")]
            print(f"{lib or '(main)'}: rc {out.returncode} reps ms {reps} {out.stderr[-300:] if out.returncode else ''}",
                  flush=True)


if __name__ == "__main__":
    main()
