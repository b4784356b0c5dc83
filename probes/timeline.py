"""Diagnostics: timeline of the last timed bench step from a rocprofv3 kernel
trace: how long the matcher ran alone, beside verification, and verification
alone, and when each matcher launch ran.  The timed steps are the trace's
longest segments (the serial isolated step, the drop-in and extraction legs
that follow them are shorter or hold no matcher-heavy work).
usage: python probes/timeline.py run_kernel_trace.csv"""
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1]))]
ev = []
for r in rows:
    n = r['Kernel_Name']
    kind = 'M' if 'match_g8_kernel' in n or 'match_tiles' in n else ('V' if 'scm::' in n else None)
    if kind:
        ev.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), kind))
ev.sort()
# last step: from the last match_tiles launch group; take the last 1/steps of match launches
mt = [e for e in ev if e[2] == 'M']
# step boundaries: gaps > 5 ms with no kernel at all
allk = sorted(ev)
segs, cur = [], [allk[0]]
for e in allk[1:]:
    if e[0] - max(x[1] for x in cur[-50:]) > 3_000_000:
        segs.append(cur)
        cur = [e]
    else:
        cur.append(e)
segs.append(cur)
print("segments:", [(round((s[-1][1] - s[0][0]) / 1e6, 1), len(s)) for s in segs])
# the last of the segments whose span is within 10 % of the longest (timed steps)
longest = max(max(e[1] for e in s) - s[0][0] for s in segs)
seg = [s for s in segs if max(e[1] for e in s) - s[0][0] >= 0.9 * longest][-1]
t0, t1 = seg[0][0], max(e[1] for e in seg)
step = 20000  # 20 us bins
nb = (t1 - t0) // step + 1
m = [0] * nb
v = [0] * nb
for s, e, k in seg:
    for b in range((s - t0) // step, (e - t0) // step + 1):
        (m if k == 'M' else v)[b] = 1
both = sum(1 for i in range(nb) if m[i] and v[i]) * step / 1e6
mo = sum(1 for i in range(nb) if m[i] and not v[i]) * step / 1e6
vo = sum(1 for i in range(nb) if v[i] and not m[i]) * step / 1e6
idle = sum(1 for i in range(nb) if not v[i] and not m[i]) * step / 1e6
print(f"step span {(t1 - t0) / 1e6:.1f} ms: match alone {mo:.1f}, both {both:.1f}, verify alone {vo:.1f}, idle {idle:.1f}")
print("matcher launches (start, end) ms:",
      [(round((s - t0) / 1e6, 1), round((e - t0) / 1e6, 1)) for s, e, k in seg if k == 'M'])
