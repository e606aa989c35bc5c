"""profiles/<round>_pmc_config2.json from the PMC passes of tools/profile.sh.

    python tools/pmc_json.py gpurun_out/prof_r4 200 2048 > profiles/r4_pmc_config2.json

The timed dispatch is the last gst_sweep_kernel launch of each pass (bench.py with
--ess-window 0 --no-stage-costs: the warmup launch, then the timed launch).  HBM bytes follow
MI355X_MICROARCH.md's gfx950 recipe: read bytes = 2 * FETCH_SIZE * 1024, write bytes =
WRITE_SIZE * 1024.
"""
import collections
import csv
import glob
import json
import sys


def last_dispatch(path, kernel="gst_sweep_kernel"):
    by = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(path)):
        if kernel in r["Kernel_Name"]:
            by[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    if not by:
        return None, {}
    d = max(by)
    return d, dict(by[d])


def main():
    root, sweeps, chains = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    ctr, disp = {}, None
    for p in ("pf", "pw", "pa", "pb", "pc"):
        for f in sorted(glob.glob(f"{root}/{p}/**/*counter_collection.csv", recursive=True)):
            d, c = last_dispatch(f)
            if c:
                disp = d
                ctr.update(c)
    rd = 2.0 * ctr["FETCH_SIZE"] * 1024
    wr = ctr["WRITE_SIZE"] * 1024
    out = {
        "source": f"rocprofv3 --pmc passes ({root}), bench.py --steps {sweeps} --warmup 20, "
                  "timed dispatch",
        "chains": chains, "sweeps": sweeps, "dispatch": disp,
        "FETCH_SIZE_KB": ctr["FETCH_SIZE"], "WRITE_SIZE_KB": ctr["WRITE_SIZE"],
        "correction": "gfx950 FETCH_SIZE reports half of wide coalesced read bytes "
                      "(MI355X_MICROARCH.md HBM): read bytes = 2*FETCH_SIZE*1024",
        "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr,
        "hbm_bytes_per_chain_sweep": (rd + wr) / (chains * sweeps),
        "record_bytes_per_chain_sweep": 3752,
        "note": "writes = the chain records (chain, bchain, zchain, alphachain, poutchain, "
                "thetachain, dfchain every sweep); T, r, sigma are L2-resident",
    }
    for k in sorted(ctr):
        if k not in ("FETCH_SIZE", "WRITE_SIZE"):
            out[k] = ctr[k]
    out["valu_active_frac_of_wave_cycles"] = ctr["SQ_ACTIVE_INST_VALU"] / ctr["SQ_WAVE_CYCLES"]
    out["lds_bank_conflict_frac_of_lds_active"] = (ctr["SQ_LDS_BANK_CONFLICT"]
                                                   / ctr["SQ_LDS_IDX_ACTIVE"])
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
