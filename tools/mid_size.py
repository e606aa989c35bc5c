"""Mid-size pulsars (missing item 2): chain-sweeps/s of the register-
resident kernel's wide TOA instances (6 / 8 slots of 64 TOAs, n <= 512) against the
large-model pipeline for the same model.

    python tools/mid_size.py [chains] [sweeps] [out.json]

Datasets: gdata.multiband epochs (J1713+0747 epochs x sub-band TOAs) under the classic
run_sims model (30 components, 14 timing-model columns), n = 260, 390, 512, 650, 910
(the last two on the 12- and 16-slot instances, round 3).
"""
import json
import sys

import numpy as np

sys.path.insert(0, ".")
from bench import CFG, initial_state  # noqa: E402
from gibbs_student_t_amd import data  # noqa: E402
from gibbs_student_t_amd.model import PTA  # noqa: E402
from gibbs_student_t_amd.native import NativeSampler  # noqa: E402


def rate(pta, C, S, path):
    ns = NativeSampler(pta, CFG, 0, path=path)
    ns.alloc(C)
    ns.set_state(**initial_state(pta, C, 0))
    ns.sweep(20, seed=1)
    ns.sweep(S, seed=1, sweep0=20)
    ns.synchronize()
    ms = ns.last_kernel_ms() if path == "persistent" else None
    stages = None
    if ms is None:
        ns.set_timing(True)
        ns.sweep(S, seed=1, sweep0=20 + S)
        ns.synchronize()
        kt = ns.kernel_times()
        ms = sum(v[0] for v in kt.values())
        stages = {k: round(v[0] / S, 4) for k, v in kt.items() if v[1]}
    ok = bool(np.all((ns.get_state()["status"] & 0xef) == 0))   # floor draws are not errors
    ns.close()
    return C * S / (ms * 1e-3), ms / S, ok, stages


def main():
    C = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    S = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    out = {"chains": C, "sweeps": S, "model": "run_sims 'beta', 30 components, 14 TM columns",
           "rows": []}
    # MS_SIZES: sub-band TOAs per J1713 epoch (130 epochs; 128 x 4 = 512); MS_PATHS: the paths
    import os
    sizes = [int(v) for v in os.environ.get("MS_SIZES", "2,3,4,5,7").split(",")]
    paths = os.environ.get("MS_PATHS", "persistent,large").split(",")
    for nsub in sizes:
        nepochs = 128 if nsub == 4 else 130
        psr = data.multiband(nepochs=nepochs, nsub=nsub, seed=7)
        pta = PTA(psr)
        for path in paths:
            r, ms, ok, stages = rate(pta, C, S if path == "persistent" else max(2, S // 10), path)
            row = {"n": pta.n, "path": path, "chain_sweeps_per_s": r, "ms_per_sweep": ms,
                   "status_clean": ok}
            if stages:
                row["stages_ms_per_sweep"] = stages
            out["rows"].append(row)
            print(json.dumps(row), flush=True)
    if len(sys.argv) > 3:
        with open(sys.argv[3], "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
