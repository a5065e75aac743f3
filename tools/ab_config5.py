"""Config 5 (bench.config5: 64M adversarial changes generated in HBM) without and with impact flags,
median ms and stage times, for A/B runs under environment switches (CORRO_OVF_SPLIT=0 ...) or library
variants (arguments: variant .so files built with corrosion_amd.build.build(out=..., defines=...),
each run in its own child process through CORRO_HIP_LIB; the in-tree library first).
    rocprofv3 --kernel-trace --stats -d gpurun_out/c5 -- python tools/ab_config5.py"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    reps = int(os.environ.get("C5_REPS", "3"))
    tag = " ".join(f"{k}={v}" for k, v in sorted(os.environ.items()) if k.startswith("CORRO_")) or "default"
    for imp in (False, True):
        ms, cells, st = bench.config5(imp, reps=reps)
        print(f"[{tag}] impact={int(imp)} ms={ms:.3f} cells={cells} stages={ {k: round(v, 3) for k, v in st.items()} }",
              flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1:
        for lib in [None] + sys.argv[1:]:
            env = dict(os.environ)
            if lib:
                env["CORRO_HIP_LIB"] = os.path.abspath(lib)
            r = subprocess.run([sys.executable, "-u", __file__], env=env, timeout=300)
            if r.returncode != 0:
                sys.exit(r.returncode)
    else:
        main()
