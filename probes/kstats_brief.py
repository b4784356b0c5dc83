"""Diagnostics: one line per kernel of a rocprofv3 kernel_stats.csv.
usage: python probes/kstats_brief.py FILE [N]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
for x in rows[:n]:
    print(f"{x['Name'][:60]:60s} {x['Calls']:>5} {float(x['AverageNs']) / 1e3:9.1f}us "
          f"{float(x['TotalDurationNs']) / 1e6:8.2f}ms {float(x['Percentage']):6.2f}")
