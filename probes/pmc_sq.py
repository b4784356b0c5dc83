"""Diagnostics: summarise SQ/GRBM PMC passes (rocprofv3 --pmc csv) of the
matcher kernels.  usage: python probes/pmc_sq.py [--kernel NAME] DIR [DIR ...] (each DIR holds
run_counter_collection.csv; the passes of one build are summed together; with
--kernel only kernels whose name contains NAME)."""
import collections
import csv
import sys


def main():
    agg = collections.defaultdict(float)
    args = sys.argv[1:]
    name = None
    if args and args[0] == "--kernel":
        name, args = args[1], args[2:]
    for d in args:
        for row in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
            if "finalize" in row["Kernel_Name"] or (name and name not in row["Kernel_Name"]):
                continue
            agg[row["Counter_Name"]] += float(row["Counter_Value"])
    w = agg["SQ_WAVE_CYCLES"] or 1.0
    out = {k: f"{v:.4g}" for k, v in sorted(agg.items())}
    print(out)
    mf = agg["SQ_INSTS_MFMA"] or 1.0
    print("wait_any %.2f wait_inst %.2f active %.2f | valu/mfma %.1f salu/mfma %.1f lds/mfma %.2f"
          % (agg["SQ_WAIT_ANY"] / w, agg["SQ_WAIT_INST_ANY"] / w, agg["SQ_ACTIVE_INST_ANY"] / w,
             agg["SQ_INSTS_VALU"] / mf, agg["SQ_INSTS_SALU"] / mf, agg["SQ_INSTS_LDS"] / mf))
    if agg.get("SQ_LDS_IDX_ACTIVE"):
        print("lds bank-conflict cycles / lds active %.3f" % (agg["SQ_LDS_BANK_CONFLICT"] / agg["SQ_LDS_IDX_ACTIVE"]))
    if agg["GRBM_GUI_ACTIVE"]:
        print("mfma busy %.3f" % (agg["SQ_VALU_MFMA_BUSY_CYCLES"] / (agg["GRBM_GUI_ACTIVE"] / 8 * 1024)))


if __name__ == "__main__":
    main()
