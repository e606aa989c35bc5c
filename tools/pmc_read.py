"""Summarise PMC passes (tools/pmc_occ.sh) of the last gst_sweep_kernel dispatch."""
import collections
import csv
import glob
import sys


def read(d, kernel="gst_sweep_kernel"):
    ctr = {}
    for f in sorted(glob.glob(f"{d}/*/*_counter_collection.csv")):
        by = collections.defaultdict(dict)
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"]:
                by[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
        if by:
            ctr.update(by[max(by)])
    return ctr


if __name__ == "__main__":
    for d in sys.argv[1:]:
        c = read(d)
        w = c.get("SQ_WAVE_CYCLES", 1)
        print(d)
        for k in sorted(c):
            print(f"  {k:28s} {c[k]:16.4g}")
        print("  -- per wave-cycle: VALU active %.3f, LDS active %.3f, any active %.3f, wait_inst %.3f, wait_any %.3f"
              % (c.get("SQ_ACTIVE_INST_VALU", 0) / w, c.get("SQ_ACTIVE_INST_LDS", 0) / w,
                 c.get("SQ_ACTIVE_INST_ANY", 0) / w, c.get("SQ_WAIT_INST_ANY", 0) / w,
                 c.get("SQ_WAIT_ANY", 0) / w))
        if "SQ_LDS_IDX_ACTIVE" in c:
            print("  -- LDS bank conflict / idx active %.3f" % (c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"]))
