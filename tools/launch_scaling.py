"""Kernel time vs sweeps per launch (fixed per-launch cost and the slowest-chain tail).

    python tools/launch_scaling.py [C]
"""
import sys

import numpy as np

sys.path.insert(0, ".")
import bench  # noqa: E402
from gibbs_student_t_amd.native import NativeSampler  # noqa: E402

C = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
wl = bench.workload(2, 0, 1, C)
ns = NativeSampler(wl["ptas"], wl["cfgs"], 0)
ns.alloc(C)
ns.set_state(**wl["init"])
ns.sweep(300, seed=1)
s0 = 300
for K in (1, 5, 10, 20, 50, 100, 200, 400):
    rec = ns.alloc_records(K, keys=("x", "b", "z", "alpha", "pout", "theta", "nu"))
    ms = []
    for rep in range(3):
        ns.sweep(K, records=rec, seed=1, sweep0=s0)
        s0 += K
        ms.append(ns.last_kernel_ms())
    print(f"K={K:4d}  kernel ms {np.median(ms):8.3f}  per sweep {np.median(ms) / K * 1e3:7.1f} us",
          flush=True)
