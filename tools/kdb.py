"""Per-kernel summary of a rocprofv3 SQLite output (run_results.db): name, calls, average and total
duration, optionally each dispatch of the named kernels in order (--each k_pk_find,...)."""
import re
import sqlite3
import sys


def short(n):
    n = re.sub(r"\(anonymous namespace\)::", "", n).replace("corro::", "").replace("void ", "")
    return "rocprim" if "rocprim" in n else n.split("(")[0]


def main():
    db = sys.argv[1]
    each = sys.argv[3].split(",") if len(sys.argv) > 3 and sys.argv[2] == "--each" else []
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, start, end from kernels order by start"))
    agg = {}
    for n, s, e in rows:
        k = short(n)
        a = agg.setdefault(k, [0, 0])
        a[0] += 1
        a[1] += e - s
    for k, (cnt, tot) in sorted(agg.items(), key=lambda x: -x[1][1])[:40]:
        print(f"{k[-60:]:60s} calls {cnt:4d} avg {tot / cnt / 1e3:10.1f} us total {tot / 1e6:9.2f} ms")
    for n, s, e in rows:
        if short(n) in each:
            print(f"  {short(n)} {(e - s) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
