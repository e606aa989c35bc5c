"""Short config-5 run of the large path for profiling (rocprofv3 -- python tools/run_large.py).

    python tools/run_large.py [sweeps] [chains] [n] [components] [ntm] [warmup sweeps]
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from bench import CFG, initial_state  # noqa: E402
from gibbs_student_t_amd import _abi, data  # noqa: E402
from gibbs_student_t_amd.model import PTA  # noqa: E402
from gibbs_student_t_amd.native import NativeSampler  # noqa: E402


def main():
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    C = int(sys.argv[2]) if len(sys.argv) > 2 else 512
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 100_000
    comp = int(sys.argv[4]) if len(sys.argv) > 4 else 60
    ntm = int(sys.argv[5]) if len(sys.argv) > 5 else 300
    if os.environ.get("RL_DATASET"):   # a golden dataset instead, e.g. RL_DATASET=ebig
        sys.path.insert(0, "tests")
        from golden_io import load_dataset
        pta = load_dataset(dataset=os.environ["RL_DATASET"])
    else:
        pta = PTA(data.scaled_synthetic(n=n, components=comp, ntm=ntm, seed=5), components=comp)
    ns = NativeSampler(pta, CFG, 0)
    ns.alloc(C)
    ns.set_state(**initial_state(pta, C, 0))
    if os.environ.get("RL_EXACT"):   # no SVD-floor pass (GST_DEBUG_EXACT_BDRAW)
        ns.set_debug(exact_bdraw=True)
    W = int(sys.argv[6]) if len(sys.argv) > 6 else 0
    if W:   # untimed warmup sweeps (the clock ramps out of idle over the first milliseconds)
        ns.sweep(W, seed=1)
        ns.synchronize()
    ns.set_timing(True)
    t0 = time.perf_counter()
    # RL_MASK: stage mask of the timed sweeps (include/gst.h), e.g. without the white MH
    mask = int(os.environ.get("RL_MASK", "0"), 0) or _abi.STAGE_ALL
    ns.sweep(S, seed=1, sweep0=W, mask=mask)
    ns.synchronize()
    dt = time.perf_counter() - t0
    kt = ns.kernel_times()
    print(f"path={ns.path} C={C} S={S} {dt / S * 1e3:.1f} ms/sweep")
    for k, (ms, nl) in kt.items():
        print(f"  {k:8s} {ms / max(1, S):9.3f} ms/sweep  ({nl} launches)")
    # status bit 4 (16): b drawn at the SVD noise floor (prior draws near log10_A = -18)
    assert np.all((ns.get_state()["status"] & 0xef) == 0)


if __name__ == "__main__":
    main()
