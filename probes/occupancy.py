"""Diagnostics: where a timed bench step's wall time goes, by the set of
kernel kinds running at each instant (rocprofv3 kernel trace).  A step bound
by total GPU work shows the wide kernels (matcher, scoring) running almost
all the time; time in which only latency-bound kernels (replay, shuffle,
draw, solve, final, finalize phases) run is time the GPU is mostly idle.
usage: python probes/occupancy.py run_kernel_trace.csv [step_index_from_end]"""
import collections
import csv
import re
import sys

WIDE = {"match", "score_F", "score_H", "exact_F", "exact_H"}


def short(name):
    m = re.search(r"scm::(\w+?)(?:<([^>]*)>)?\(", name)
    if not m:
        return name.split("(")[0][-30:]
    base, targ = m.group(1), m.group(2) or ""
    base = base.replace("_kernel", "")
    if base.startswith("match_g8") or base.startswith("match_tiles"):
        return "match"
    if base == "rs_score":
        return "score_" + ("F" if targ.startswith("0") or "KIND_F" in targ else "H")
    if base == "rs_exact":
        return "exact_" + ("F" if targ.startswith("0") or "KIND_F" in targ else "H")
    if base.startswith("rs_solve"):
        return "solve_" + ("F" if targ.startswith("0") or "KIND_F" in targ else "H")
    return base


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    which = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                 int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"])), int(r["VGPR_Count"]))
                for r in rows if "scm::" in r["Kernel_Name"])
    # steps: segments separated by > 3 ms with no kernel
    segs, cur, end = [], [ev[0]], ev[0][1]
    for e in ev[1:]:
        if e[0] - end > 3_000_000:
            segs.append(cur)
            cur = [e]
        else:
            cur.append(e)
        end = max(end, e[1])
    segs.append(cur)
    spans = [max(e[1] for e in s) - s[0][0] for s in segs]
    longest = max(spans)
    steps = [s for s, sp in zip(segs, spans) if sp >= 0.8 * longest and any(e[2] == "match" for e in s)]
    seg = steps[-which]
    t0, t1 = seg[0][0], max(e[1] for e in seg)
    print(f"segments (ms): {[round(sp / 1e6, 1) for sp in spans]}; step {len(steps) - which} of "
          f"{len(steps)}: {(t1 - t0) / 1e6:.1f} ms, {len(seg)} kernels")
    # sweep over start / end points
    pts = sorted({x for e in seg for x in (e[0], e[1])})
    by_sig = collections.Counter()
    by_kind = collections.Counter()
    narrow_only = 0
    import bisect
    starts = [e[0] for e in seg]
    for a, b in zip(pts, pts[1:]):
        mid = (a + b) / 2
        act = sorted({e[2] for e in seg[:bisect.bisect_right(starts, mid)] if e[0] <= mid < e[1]})
        by_sig[" + ".join(act) if act else "(idle)"] += b - a
        for k in act:
            by_kind[k] += b - a
        if act and not (set(act) & WIDE):
            narrow_only += b - a
    tot = t1 - t0
    print(f"time with only latency-bound kernels: {narrow_only / 1e6:.1f} ms "
          f"({100 * narrow_only / tot:.0f} %)")
    print("kernel kinds, time active (ms; overlapping):")
    for k, v in by_kind.most_common():
        print(f"  {k:28s} {v / 1e6:7.1f}")
    print("instants by running set (ms):")
    for k, v in by_sig.most_common(25):
        print(f"  {v / 1e6:7.1f}  {k}")
    # launch geometry of the latency-bound kinds
    geo = collections.defaultdict(list)
    for e in seg:
        geo[e[2]].append((e[3], e[4], e[1] - e[0]))
    print("launches: kind, count, blocks (min-max), VGPRs, mean / max ms")
    for k, v in sorted(geo.items()):
        print(f"  {k:28s} {len(v):4d} {min(x[0] for x in v):6d}-{max(x[0] for x in v):6d} "
              f"{v[0][1]:4d} {sum(x[2] for x in v) / len(v) / 1e6:7.3f} {max(x[2] for x in v) / 1e6:7.3f}")


if __name__ == "__main__":
    main()
