"""Diagnostics: per-kernel totals of one or more rocprofv3 kernel_stats.csv files, side by side.
usage: python probes/kstats.py DIV file1.csv [file2.csv ...]   (DIV: divide totals, e.g. steps)"""
import csv
import sys

div = float(sys.argv[1])
tabs = []
for f in sys.argv[2:]:
    t = {}
    for r in csv.DictReader(open(f)):
        t[r['Name'].split('(')[0].replace('void ', '').replace('scm::', '')[:34]] = (
            int(r['TotalDurationNs']) / 1e6 / div, int(r['Calls']))
    tabs.append(t)
names = sorted(tabs[0], key=lambda n: -tabs[0][n][0])
for n in names:
    print(f"{n:35s}" + "".join(f" {t.get(n, (0, 0))[0]:9.2f}ms {t.get(n, (0, 0))[1]:5d}" for t in tabs))
print(f"{'TOTAL':35s}" + "".join(f" {sum(v[0] for v in t.values()):9.2f}ms" for t in tabs))
