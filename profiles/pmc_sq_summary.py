#!/usr/bin/env python3
"""Summarise rocprofv3 SQ / GRBM PMC passes of bench.py per kernel.

usage: pmc_sq_summary.py OUT_JSON DIR [DIR ...] [--kernel NAME=PATTERN ...]

Each DIR holds one pass's run_counter_collection.csv (counters that cannot
share a pass come from separate runs of the same command).  Per kernel: the
per-launch counter values (mean over its dispatches), VALU instructions per
MFMA, MFMA busy and VALU-active fractions of the chip's SIMD cycles
(GRBM_GUI_ACTIVE counts the GPU clock once per XCD: x 1024 SIMDs / 8 XCDs;
SQ_ACTIVE_INST_VALU is in quad-cycles: x 4),
and the wave-cycle split (waiting on anything / on an instruction dependency /
issuing)."""
import argparse
import collections
import csv
import json

DEFAULT = {
    "match_g8_kernel": "match_g8_kernel",
    "rs_score_kernel<1>": "rs_score_kernel<1",
    "rs_score_kernel<0>": "rs_score_kernel<0",
    "rs_replay2_kernel": "rs_replay2_kernel",
}


def lib_sha(v):
    """bench.py uses a summary only when this hash equals the loaded library's."""
    import os
    if v and os.path.exists(v):
        return open(v).read().split()[0][:16]
    return v


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out_json")
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--kernel", action="append", default=[])
    ap.add_argument("--lib-sha16", default=None,
                    help="sha256[:16] of the libscm.so the profiled run loaded (or a file holding it)")
    a = ap.parse_args()
    kernels = dict(k.split("=", 1) for k in a.kernel) if a.kernel else DEFAULT
    out = {}
    for name, pat in kernels.items():
        sums = collections.defaultdict(float)
        disp = collections.defaultdict(set)
        for d in a.dirs:
            for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
                if pat not in r["Kernel_Name"]:
                    continue
                sums[r["Counter_Name"]] += float(r["Counter_Value"])
                disp[r["Counter_Name"]].add((d, r["Dispatch_Id"]))
        if not sums:
            continue
        per = {c: v / max(1, len(disp[c])) for c, v in sorted(sums.items())}
        n = max(len({i for _, i in s}) for s in disp.values())
        simd = per.get("GRBM_GUI_ACTIVE", 0.0) / 8 * 1024
        w = per.get("SQ_WAVE_CYCLES", 0.0)
        mf = per.get("SQ_INSTS_MFMA", 0.0)
        out[name] = {
            "dispatches": n,
            "per_launch": per,
            "valu_per_mfma": per["SQ_INSTS_VALU"] / mf if mf and "SQ_INSTS_VALU" in per else None,
            "mfma_busy": (per["SQ_VALU_MFMA_BUSY_CYCLES"] / simd
                          if simd and "SQ_VALU_MFMA_BUSY_CYCLES" in per else None),
            "valu_active_frac_of_simd_cycles": (4 * per["SQ_ACTIVE_INST_VALU"] / simd
                                                if simd and "SQ_ACTIVE_INST_VALU" in per else None),
            "wave_cycle_split": ({"wait_any": per.get("SQ_WAIT_ANY", 0.0) / w,
                                  "wait_inst_any": per.get("SQ_WAIT_INST_ANY", 0.0) / w,
                                  "active_inst_any": per.get("SQ_ACTIVE_INST_ANY", 0.0) / w}
                                 if w else None),
        }
    out["lib_sha16"] = lib_sha(a.lib_sha16)
    json.dump(out, open(a.out_json, "w"), indent=1)
    for k, v in out.items():
        if not isinstance(v, dict):
            continue
        print(k, v["dispatches"], {x: v[x] for x in ("valu_per_mfma", "mfma_busy",
                                                     "valu_active_frac_of_simd_cycles")})


if __name__ == "__main__":
    main()
