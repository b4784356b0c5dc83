"""Diagnostics: per-stream activity of the last bench step in a rocprofv3 kernel trace.
usage: python probes/streams.py run_kernel_trace.csv"""
import collections
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1]))]
ev = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']),
             r['Kernel_Name'].split('(')[0].replace('void ', '').replace('scm::', ''), r['Stream_Id'])
            for r in rows)
# step starts: a match_tiles launch after >3 ms with no kernel running
starts, end = [], 0
for s, e, n, st in ev:
    if s - end > 3_000_000 and 'match_tiles' in n:
        starts.append(s)
    end = max(end, e)
t0 = starts[-1]
last = [x for x in ev if x[0] >= t0]
by = collections.defaultdict(list)
for s, e, n, st in last:
    by[st].append((s, e, n))
for k, v in sorted(by.items(), key=lambda kv: kv[1][0][0]):
    busy = sum(e - s for s, e, n in v)
    mts = [(s, e) for s, e, n in v if 'match_tiles' in n]
    extra = " match_tiles " + ", ".join(f"[{(s - t0) / 1e6:.0f}-{(e - t0) / 1e6:.0f}]" for s, e in mts) if mts else ""
    vb = [(s, e) for s, e, n in v if 'rs_begin_kernel<0>' in n or 'verify_final' in n]
    extra += " verify " + ", ".join(f"{(s - t0) / 1e6:.0f}" for s, e in vb) if vb else ""
    print(f"stream {k}: start {(v[0][0] - t0) / 1e6:6.1f} end {(max(e for s, e, n in v) - t0) / 1e6:6.1f} "
          f"busy {busy / 1e6:6.1f} n={len(v)}{extra}")
print(f"step GPU span {(max(e for s, e, n, st in last) - t0) / 1e6:.1f} ms")
