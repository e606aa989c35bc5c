"""profiles/pmc_traffic.json from the PMC passes of tools/profile_config2.sh.

    python tools/pmc_config2.py <prof_dir> <sweeps> <chains> > profiles/pmc_traffic.json

The timed dispatch is the last gst_sweep_kernel launch of each pass (bench.py: warmup
launch, then the timed launch).  HBM bytes follow MI355X_MICROARCH.md's gfx950 recipe:
FETCH_SIZE reports half of wide coalesced read bytes, so read bytes = 2 * FETCH_SIZE KB.
"""
import collections
import csv
import glob
import json
import os
import sys


def timed(path):
    by = collections.defaultdict(dict)
    for r in csv.DictReader(open(path)):
        if "gst_sweep_kernel" in r["Kernel_Name"]:
            by[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    if not by:          # a pass of another workload (e.g. config 5 in the same directory)
        return None, {}
    last = max(by)
    return last, by[last]


def main():
    d, sweeps, chains = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    out = {"source": f"rocprofv3 --pmc passes ({d}), bench.py --steps {sweeps} --warmup 20, "
                     "timed dispatch", "chains": chains, "sweeps": sweeps}
    ctr = {}
    for f in sorted(glob.glob(os.path.join(d, "*", "*_counter_collection.csv"))):
        disp, c = timed(f)
        if disp is None:
            continue
        ctr.update(c)
        out.setdefault("dispatch", disp)
    rd = 2.0 * ctr["FETCH_SIZE"] * 1024
    wr = ctr["WRITE_SIZE"] * 1024
    out.update({
        "FETCH_SIZE_KB": ctr["FETCH_SIZE"], "WRITE_SIZE_KB": ctr["WRITE_SIZE"],
        "correction": "gfx950 FETCH_SIZE reports half of wide coalesced read bytes "
                      "(MI355X_MICROARCH.md HBM): read bytes = 2*FETCH_SIZE*1024",
        "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr,
        "hbm_bytes_per_chain_sweep": (rd + wr) / (sweeps * chains),
        "record_bytes_per_chain_sweep": 8 * (3 + 74 + 3 * 130 + 2),
        "note": "writes = the chain records (chain, bchain, zchain, alphachain, poutchain, "
                "thetachain, dfchain every sweep); T, r, sigma are L2-resident",
    })
    for k in sorted(ctr):
        if k not in ("FETCH_SIZE", "WRITE_SIZE"):
            out[k] = ctr[k]
    if "SQC_ICACHE_HITS" in ctr:
        out["icache_miss_rate"] = ctr["SQC_ICACHE_MISSES"] / (ctr["SQC_ICACHE_HITS"] +
                                                              ctr["SQC_ICACHE_MISSES"])
    if "SQ_ACTIVE_INST_VALU" in ctr:
        out["valu_active_frac_of_wave_cycles"] = ctr["SQ_ACTIVE_INST_VALU"] / ctr["SQ_WAVE_CYCLES"]
        out["lds_bank_conflict_frac_of_lds_active"] = (ctr["SQ_LDS_BANK_CONFLICT"] /
                                                       ctr["SQ_LDS_IDX_ACTIVE"])
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
