"""Diagnostics: the kernel/copy timeline of one drop-in call from a rocprofv3
kernel trace (a call = from its matcher launch to the next call's).
usage: python probes/call_timeline.py TRACE.csv [CALL]"""
import csv
import sys

r = list(csv.DictReader(open(sys.argv[1])))
r.sort(key=lambda x: int(x['Start_Timestamp']))
call = int(sys.argv[2]) if len(sys.argv) > 2 else 4
idx = [i for i, x in enumerate(r) if 'match_g8_kernel' in x['Kernel_Name']]
a, b = idx[call], idx[call + 1]
t0 = int(r[a]['Start_Timestamp'])
prev_end = t0
busy = 0
for x in r[a:b]:
    s, e = int(x['Start_Timestamp']), int(x['End_Timestamp'])
    busy += e - s
    print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:8.1f} gap {(s - prev_end) / 1e3:7.1f}  {x['Kernel_Name'][:60]}")
    prev_end = max(prev_end, e)
print(f"span {(prev_end - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us")
