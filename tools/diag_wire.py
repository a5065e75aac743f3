"""Phase times of k_wire_decode (CORRO_DIAG 512 variant, tools/_variants/libcorro_wdiag.so):
staging, wave walk and per-lane decode of every 997th frame, printed by the kernel."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

if __name__ == "__main__":
    lib = os.path.join(ROOT, "tools", "_variants", "libcorro_wdiag.so")
    if "--build" in sys.argv:
        from corrosion_amd import build
        build.build(out=lib, defines=["-DCORRO_DIAG=512"])
        sys.exit(0)
    env = dict(os.environ, CORRO_HIP_LIB=lib)
    sys.exit(subprocess.call([sys.executable, os.path.join(ROOT, "bench_wire.py"), "--steps", "1", "--warmup", "1"],
                             env=env))
