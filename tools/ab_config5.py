"""Config 5 (bench.config5: 64M adversarial changes generated in HBM) without and with impact flags,
median ms and stage times, for A/B runs under environment switches (CORRO_OVF_SPLIT=0 ...).
    rocprofv3 --kernel-trace --stats -d gpurun_out/c5 -- python tools/ab_config5.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import bench
    reps = int(os.environ.get("C5_REPS", "3"))
    tag = " ".join(f"{k}={v}" for k, v in sorted(os.environ.items()) if k.startswith("CORRO_")) or "default"
    for imp in (False, True):
        ms, cells, st = bench.config5(imp, reps=reps)
        print(f"[{tag}] impact={int(imp)} ms={ms:.3f} cells={cells} stages={ {k: round(v, 3) for k, v in st.items()} }",
              flush=True)


if __name__ == "__main__":
    main()
