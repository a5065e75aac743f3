"""Summarise a gpurun_out/prof directory (scripts/gpu.sh) into a markdown table:
per-kernel average duration (rocprofv3 --kernel-trace --stats) and HBM traffic per dispatch from
the separate --pmc passes: 2 x FETCH_SIZE (gfx950 reports half of wide coalesced reads,
MI355X_MICROARCH.md §HBM) + WRITE_SIZE, both in KiB.

python tools/prof_summary.py gpurun_out/prof > profiles/rNN_summary.md
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def kname(n):
    return n.split("(")[0].replace("void ", "").strip()


def stats(path):
    out = {}
    for r in csv.DictReader(open(path)):
        if "corro" in r["Name"]:
            out[kname(r["Name"])] = (int(r["Calls"]), float(r["AverageNs"]) / 1e3)
    return out


def pmc(path, counter):
    tot, disp = defaultdict(float), defaultdict(set)
    for r in csv.DictReader(open(path)):
        if "corro" in r["Kernel_Name"] and r["Counter_Name"] == counter:
            k = kname(r["Kernel_Name"])
            tot[k] += float(r["Counter_Value"])
            disp[k].add(r["Dispatch_Id"])
    return {k: tot[k] / len(disp[k]) * 1024.0 for k in tot}


def section(title, d, trace, fetch, write):
    st = stats(os.path.join(d, trace, "run_kernel_stats.csv"))
    fe = pmc(os.path.join(d, fetch, "run_counter_collection.csv"), "FETCH_SIZE") if fetch else {}
    wr = pmc(os.path.join(d, write, "run_counter_collection.csv"), "WRITE_SIZE") if write else {}
    print(f"### {title}\n")
    print("| kernel | calls | avg µs | HBM read GB (2×FETCH) | HBM write GB | GB/s from PMC |")
    print("|---|---|---|---|---|---|")
    for k, (c, us) in sorted(st.items(), key=lambda x: -x[1][1]):
        r = 2 * fe.get(k, 0.0) / 1e9
        w = wr.get(k, 0.0) / 1e9
        bw = (r + w) / (us * 1e-6) if us > 0 else 0.0
        print(f"| {k} | {c} | {us:.1f} | {r:.3f} | {w:.3f} | {bw:.0f} |")
    print()


def main():
    d = sys.argv[1]
    section("config 2 merge pipeline (bench.py --steps 3 --warmup 1)", d, "trace", "pmc_FETCH_SIZE", "pmc_WRITE_SIZE")
    if os.path.isdir(os.path.join(d, "sync_trace")):
        section("config 4 sync-need diff (bench_sync.py --steps 3 --warmup 1)", d, "sync_trace", "sync_pmc_FETCH",
                "sync_pmc_WRITE")


if __name__ == "__main__":
    main()
