"""Stage cycles of the driver's timed window (20 sweeps right after 5 warmup sweeps from the
bench's initial state) vs the same window after burn-in: which stage makes early sweeps slow?
    GST_LIB=gibbs_student_t_amd/libgst_stamps.so python tools/diag/early_profile.py"""
import ctypes as ct
import sys

import numpy as np
import torch

import os  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import bench  # noqa: E402
from gibbs_student_t_amd import _abi  # noqa: E402
from gibbs_student_t_amd.native import NativeSampler  # noqa: E402
from stage_profile import STAGES  # noqa: E402

C, K = 2048, 20
wl = bench.workload(2, 0, 1, C)
ns = NativeSampler(wl["ptas"], wl["cfgs"], 0)
ns.alloc(C)
ns.set_state(**wl["init"])
ns.sweep(5, seed=1)
buf = torch.zeros((C, 20), dtype=torch.int64, device=ns.tdev)
s0 = 5
for tag, pre in (("early (after 5)", 0), ("after +1000", 1000)):
    if pre:
        ns.sweep(pre, seed=1, sweep0=s0)
        s0 += pre
        ns.sweep(20, seed=1, sweep0=s0)   # let the clock recover after the long launch
        s0 += 20
    buf.zero_()
    _abi.check(ns.lib, ns.lib.gst_debug_stamps(ns.ctx, ct.c_void_p(buf.data_ptr())), "st")
    ns.sweep(K, seed=1, sweep0=s0)
    ns.synchronize()
    s0 += K
    _abi.check(ns.lib, ns.lib.gst_debug_stamps(ns.ctx, ct.c_void_p(0)), "st")
    cyc = buf.cpu().numpy().astype(np.float64) / K
    tot = cyc[:, :7].sum(axis=1)
    w = int(np.argmax(tot))
    print(f"== {tag}: kernel {ns.last_kernel_ms() / K * 1e3:.1f} us/sweep; per-chain mean {tot.mean():.0f} "
          f"max {tot.max():.0f} (chain {w})")
    for i, nm in enumerate(STAGES):
        print(f"  {nm:24s} mean {cyc[:, i].mean():9.0f}  slowest chain {cyc[w, i]:9.0f}")
    for i, nm in ((16, "lnL evals"), (18, "accepted hyper")):
        print(f"  {nm:24s} mean {cyc[:, i].mean():9.2f}  slowest chain {cyc[w, i]:9.2f}")
