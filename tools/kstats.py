import csv, glob, re, sys
fs = sorted(glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True))
for r in csv.DictReader(open(fs[-1])):
    print("%-60s calls %4s avg %10.1f us  total %9.2f ms" % (re.sub(r'\(anonymous namespace\)::', '', r['Name']).split('(')[0][-60:], r['Calls'], float(r['AverageNs'])/1e3, float(r['TotalDurationNs'])/1e6))
