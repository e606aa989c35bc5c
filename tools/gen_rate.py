"""Chain-sweeps/s of the general white-noise model (per-backend efac / equad, ECORR) on the
persistent kernel's GEN instances against the large path, same dataset and start.

    python tools/gen_rate.py [sweeps] [datasets]     e.g. python tools/gen_rate.py 200 ecb,ecq
    (GR_PATHS=large: the large path only, e.g. for ebig's 150-column red-noise / ECORR block;
     GR_DEBUG=epochs_lds[,...]: NativeSampler.set_debug flags;
     GR_STAGES=1: the large path's per-stage ms per sweep over S further timed sweeps)

Datasets are the golden ones (tests/golden/<name>_dataset.npz); the model is bench.py's
(outlier mixture, beta theta prior, varied nu), chains start from prior draws.
"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from bench import CFG, initial_state  # noqa: E402
from golden_io import load_dataset  # noqa: E402
from gibbs_student_t_amd.native import NativeSampler  # noqa: E402


def rate(pta, path, C, S, W=20):
    ns = NativeSampler(pta, CFG, 0, path=path)
    if os.environ.get("GR_DEBUG"):      # e.g. GR_DEBUG=epochs_lds (A/B of a kernel choice)
        ns.set_debug(**{k: True for k in os.environ["GR_DEBUG"].split(",")})
    ns.alloc(C)
    ns.set_state(**initial_state(pta, C, 0))
    ns.sweep(W, seed=3)
    ns.synchronize()
    t0 = time.perf_counter()
    ns.sweep(S, seed=3, sweep0=W)
    ns.synchronize()
    dt = time.perf_counter() - t0
    ok = bool(np.all((ns.get_state()["status"] & 0xef) == 0))
    stages = None
    if path == "large" and os.environ.get("GR_STAGES"):
        ns.set_timing(True)
        ns.sweep(S, seed=3, sweep0=W + S)
        ns.synchronize()
        stages = {k: round(v[0] / S, 5) for k, v in ns.kernel_times().items() if v[1]}
    ns.close()
    return C * S / dt, ok, stages


def main():
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    names = (sys.argv[2] if len(sys.argv) > 2 else "ecb,ecq,jb").split(",")
    out = []
    for nm in names:
        pta = load_dataset(dataset=nm)
        for C in (512, 2048):
            for path in os.environ.get("GR_PATHS", "persistent,large").split(","):
                r, ok, stages = rate(pta, path, C, S)
                row = dict(dataset=nm, n=pta.n, m=pta.m, P=len(pta.params), chains=C, path=path,
                           sweeps=S, chain_sweeps_per_s=r, status_ok=ok)
                if stages:
                    row["stages_ms_per_sweep"] = stages
                print(json.dumps(row), flush=True)
                out.append(row)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
