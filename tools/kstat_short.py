"""Per-apply kernel summary of a rocprofv3 kernel_stats.csv (rocPRIM names shortened).
python tools/kstat_short.py <kernel_stats.csv> <applies>"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
applies = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
for x in rows:
    n = x["Name"]
    m = re.search(r"(radix_sort_onesweep_\w+|scan_by_key_impl|init_device_scan_by_key_kernel|scan_impl\w*|lookback_scan\w*)", n)
    tag = m.group(1) if m else n[:60]
    if "rocprim" in n:
        m2 = re.search(r"default_config, ([\w:<> ]+?), ([\w:<> ]+?)>", n)
        tag += " " + (m2.group(1) + "," + m2.group(2) if m2 else "")
    print(f"{tag[:80]:80s} {x['Calls']:>5} {float(x['AverageNs'])/1e3:10.1f} us  {float(x['TotalDurationNs'])/1e6/applies:8.2f} ms/apply")
