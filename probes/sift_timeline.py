"""Timeline of an extraction kernel trace (rocprofv3 --kernel-trace csv): the
last call's frames (a call starts at the first upsample_kernel after a gap),
per-frame chain time, GPU busy union, and per-kernel time by octave.
usage: python probes/sift_timeline.py run_kernel_trace.csv [frames_per_call]"""
import csv
import sys
from collections import defaultdict

path = sys.argv[1]
fpc = int(sys.argv[2]) if len(sys.argv) > 2 else 16
rows = [r for r in csv.DictReader(open(path))]
ks = []
for r in rows:
    name = r["Kernel_Name"].replace("(anonymous namespace)", "anon").split("(")[0].split("::")[-1]
    ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, int(r["Queue_Id"]),
               int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])))
ks.sort()
ups = [i for i, k in enumerate(ks) if k[2] == "upsample_kernel"]
# the last call: its fpc upsamples
first = ups[-fpc]
sel = ks[first:]
t0 = sel[0][0]
t1 = max(k[1] for k in sel)
print(f"last call: {len(sel)} kernels, {(t1 - t0) / 1e3:.1f} us first-upsample -> last end "
      f"({(t1 - t0) / 1e3 / fpc:.1f} us per frame)")
# busy union
iv = sorted((k[0], k[1]) for k in sel)
busy, cs, ce = 0, iv[0][0], iv[0][1]
for s, e in iv[1:]:
    if s > ce:
        busy += ce - cs
        cs, ce = s, e
    else:
        ce = max(ce, e)
busy += ce - cs
print(f"GPU busy union {busy / 1e3:.1f} us ({busy / (t1 - t0):.2f} of the span)")
# per-kernel sums and the octave of each descriptor launch (4 per frame, in order per queue)
tot = defaultdict(float)
cnt = defaultdict(int)
for k in sel:
    tot[k[2]] += (k[1] - k[0]) / 1e3
    cnt[k[2]] += 1
for n, v in sorted(tot.items(), key=lambda x: -x[1])[:12]:
    print(f"  {n:28s} {cnt[n]:5d} launches {v:9.1f} us sum  {v / cnt[n]:8.1f} us avg")
# frames: per queue, chains from upsample to the fixup
byq = defaultdict(list)
for k in sel:
    byq[k[3]].append(k)
for q, lst in sorted(byq.items()):
    frames, cur = [], None
    for k in lst:
        if k[2] == "upsample_kernel":
            cur = [k]
            frames.append(cur)
        elif cur is not None:
            cur.append(k)
    for f in frames:
        d = [(k[1] - k[0]) / 1e3 for k in f if k[2] == "descriptor_kernel"]
        o = [(k[1] - k[0]) / 1e3 for k in f if k[2] == "orient_kernel"]
        kern = sum((k[1] - k[0]) for k in f) / 1e3
        print(f"queue {q}: frame span {(f[-1][1] - f[0][0]) / 1e3:8.1f} us, kernels {kern:8.1f} us, "
              f"descriptor by octave {['%.0f' % x for x in d]}, orient {['%.0f' % x for x in o]}, "
              f"start {(f[0][0] - t0) / 1e3:.0f}")
