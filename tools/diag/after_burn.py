"""20-sweep launches right after a long burn-in launch (the driver's timed region follows
bench.py's 3000-sweep burn-in): is the first one slower, and why?"""
import sys
import time

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from gibbs_student_t_amd.native import NativeSampler  # noqa: E402

C, K = 2048, 20
wl = bench.workload(2, 0, 1, C)
ns = NativeSampler(wl["ptas"], wl["cfgs"], 0)
ns.alloc(C)
ns.set_state(**wl["init"])
keys = ("x", "b", "z", "alpha", "pout", "theta", "nu")
s0 = 0


def run(n, rec=None):
    global s0
    ns.sweep(n, records=rec, seed=1, sweep0=s0)
    ns.synchronize()
    s0 += n
    return ns.last_kernel_ms() / n * 1e3


ns.sweep(5, seed=1)
s0 = 5
for burn in (3000, 300, 3000):
    b = run(burn)
    rec = ns.alloc_records(K, keys)
    t = [run(K, rec) for _ in range(4)]
    print(f"burn {burn} ({b:.1f} us/sweep) then 20-sweep launches: " + " ".join(f"{x:.1f}" for x in t), flush=True)
b = run(3000)
time.sleep(0.5)
t = [run(K, rec) for _ in range(3)]
print(f"burn 3000 ({b:.1f}), 0.5 s idle, then: " + " ".join(f"{x:.1f}" for x in t), flush=True)
b = run(3000)
t = [run(K, rec) for _ in range(3)] + [run(500, ns.alloc_records(500, keys))]
print(f"burn 3000 ({b:.1f}), then 20,20,20,500: " + " ".join(f"{x:.1f}" for x in t), flush=True)

# with the diagnostic stamps library: implied shader clock = slowest chain's cycles / kernel time
import ctypes as ct  # noqa: E402
import os  # noqa: E402

import numpy as np  # noqa: E402

from gibbs_student_t_amd import _abi  # noqa: E402

if "stamps" in os.environ.get("GST_LIB", ""):
    buf = torch.zeros((C, 20), dtype=torch.int64, device=ns.tdev)
    for burn in (3000, 300):
        run(burn)
        out = []
        for _ in range(4):
            buf.zero_()
            _abi.check(ns.lib, ns.lib.gst_debug_stamps(ns.ctx, ct.c_void_p(buf.data_ptr())), "st")
            us = run(K, rec)
            cyc = buf.cpu().numpy().astype(np.float64)[:, :7].sum(axis=1) / K
            out.append(f"{us:.1f}us max {cyc.max():.0f}cyc clk {cyc.max() / us / 1e3:.3f}GHz")
            _abi.check(ns.lib, ns.lib.gst_debug_stamps(ns.ctx, ct.c_void_p(0)), "st")
        print(f"burn {burn}: " + " | ".join(out), flush=True)
