"""Per-kernel summary of rocprofv3 CSV outputs: kernel-trace stats + separate --pmc passes.

    python tools/pmc_summary.py <kernel_stats.csv> <out.json> <counter_collection.csv> ...

For every kernel: average launch duration (kernel stats), per-dispatch averages of the
counters collected, and the derived HBM bytes (gfx950: read bytes = 2 x FETCH_SIZE x 1024,
MI355X_MICROARCH.md HBM section; write bytes = WRITE_SIZE x 1024), HBM GB/s and executed
fp64 MFMA work (SQ_INSTS_VALU_MFMA_MOPS_F64 x 512 flop).
"""
from __future__ import annotations

import csv
import json
import re
import sys
from collections import defaultdict

HBM_PEAK_GBS = 8000.0
FP64_PEAK_TFLOPS = 78.6


def short(name: str) -> str:
    m = re.search(r"gst::(\w+)", name)
    return m.group(1) if m else name.split("(")[0]


def main():
    stats_csv, out_json, *pmc_csvs = sys.argv[1:]
    avg_ms = {}
    for r in csv.DictReader(open(stats_csv)):
        avg_ms[short(r["Name"])] = float(r["AverageNs"]) / 1e6
    ctr = defaultdict(lambda: defaultdict(list))
    for f in pmc_csvs:
        for r in csv.DictReader(open(f)):
            ctr[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    kernels = {}
    for k in sorted(set(avg_ms) | set(ctr)):
        d = {"avg_ms": avg_ms.get(k)}
        c = {n: sum(v) / len(v) for n, v in ctr[k].items()}
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            d["hbm_read_bytes"] = 2.0 * c["FETCH_SIZE"] * 1024
            d["hbm_write_bytes"] = c["WRITE_SIZE"] * 1024
            if d["avg_ms"]:
                gbs = (d["hbm_read_bytes"] + d["hbm_write_bytes"]) / (d["avg_ms"] * 1e-3) / 1e9
                d["hbm_GBps"] = gbs
                d["hbm_frac"] = gbs / HBM_PEAK_GBS
        if c.get("SQ_INSTS_VALU_MFMA_MOPS_F64"):
            d["mfma_f64_executed_flop"] = c["SQ_INSTS_VALU_MFMA_MOPS_F64"] * 512
            if d["avg_ms"]:
                d["mfma_f64_executed_TFLOPs"] = d["mfma_f64_executed_flop"] / (d["avg_ms"] * 1e-3) / 1e12
        for n in ("SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                  "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE"):
            if n in c:
                d[n] = c[n]
        kernels[k] = d
    out = {"source": "rocprofv3 --kernel-trace --stats and separate --pmc passes; per-launch "
                     "averages (" + ", ".join(sys.argv[1:]) + ")",
           "correction": "HBM read bytes = 2 x FETCH_SIZE x 1024 (MI355X_MICROARCH.md gfx950 "
                         "FETCH_SIZE); write bytes = WRITE_SIZE x 1024",
           "hbm_peak_GBps": HBM_PEAK_GBS, "fp64_peak_TFLOPs": FP64_PEAK_TFLOPS,
           "kernels": kernels}
    with open(out_json, "w") as f:
        json.dump(out, f, indent=1)
    for k, d in kernels.items():
        print(k, {a: (round(b, 3) if isinstance(b, float) else b) for a, b in d.items()
                  if a in ("avg_ms", "hbm_GBps", "mfma_f64_executed_TFLOPs")})


if __name__ == "__main__":
    main()
