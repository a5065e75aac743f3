"""Build libcorro_hip.so in-tree with hipcc for gfx950 (no JIT cache, no pip install).

python -m corrosion_amd.build  [--force]
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libcorro_hip.so")
SOURCES = ["engine.hip", "sync_needs.hip", "partition.hip", "prims.hip", "extract.hip", "wire.hip", "booked.cpp", "agent.cpp",
           "pkeys.hip", "gaps.hip", "affinity.hip", "agent_dev.hip", "bufpool.hip"]
HEADERS = ["internal.h", "merge_kernels.h", "ovf_kernels.h", "ranges.h", "booked.h", "rowhash.h", "rowstore.h", "agent_dev.h"]
ARCH = "gfx950"


FLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function", f"--offload-arch={ARCH}"]
STAMP = LIB + ".srchash"


def _source_hash():
    """sha256 over every source, header and the build flags: the library is rebuilt when any of
    them changes, whatever the files' mtimes (a copied tree keeps a valid build)."""
    import hashlib
    h = hashlib.sha256(" ".join(FLAGS + SOURCES).encode())
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS] + [os.path.join(ROOT, "include", "corro_hip.h")]
    for d in deps:
        with open(d, "rb") as f:
            h.update(os.path.basename(d).encode() + b"\0" + f.read())
    return h.hexdigest()


def _stale():
    if not os.path.exists(LIB) or not os.path.exists(STAMP):
        return True
    with open(STAMP) as f:
        return f.read().strip() != _source_hash()


def build(force=False, verbose=False, out=None, defines=()):
    """Build LIB (or, with `out`/`defines`, a variant of it at `out`: diagnostics only)."""
    if out is not None:
        return _build_to(out, list(defines), verbose)
    if not force and not _stale():
        return LIB
    return _build_to(LIB, [], verbose, stamp=True)


def _build_to(lib, defines, verbose, stamp=False):
    src_hash = _source_hash()  # of the sources this build compiles (not of later edits)
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    from concurrent.futures import ThreadPoolExecutor
    jobs = []
    objs = []
    for src in SOURCES:
        obj = os.path.join(os.path.dirname(lib), os.path.basename(lib) + "." + src + ".o")
        # (-Wno-unused-function: the host pass of a .hip file reports the static kernels of a shared
        # header that the file does not launch itself)
        cmd = [hipcc] + FLAGS + defines + ["-I", os.path.join(ROOT, "include"), "-I", CSRC, "-c", os.path.join(CSRC, src),
                                 "-o", obj]
        if src.endswith(".cpp"):
            cmd = [hipcc, "-O3", "-std=c++17", "-fPIC", "-Wall", "-x", "c++",
                   "-I", os.path.join(ROOT, "include"), "-I", CSRC, "-c", os.path.join(CSRC, src), "-o", obj]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        jobs.append(cmd)
        objs.append(obj)
    workers = max(1, min(len(jobs), int(os.environ.get("MAX_JOBS") or os.cpu_count() or 1)))
    with ThreadPoolExecutor(workers) as ex:
        for f in [ex.submit(subprocess.check_call, c) for c in jobs]:
            f.result()
    tmp = lib + ".tmp"
    subprocess.check_call([hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", tmp] + objs)
    os.replace(tmp, lib)
    for o in objs:
        os.remove(o)
    if stamp:
        with open(STAMP, "w") as f:
            f.write(src_hash)
    return lib


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
    print(LIB)
