"""Spread of per-chain sweep time (diagnostic libgst_stamps.so): why a short launch runs
slower per sweep than a long one -- the kernel ends with its slowest chain.

    GST_LIB=gibbs_student_t_amd/libgst_stamps.so python tools/chain_spread.py [C]
"""
import ctypes as ct
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from gibbs_student_t_amd import _abi  # noqa: E402
from gibbs_student_t_amd.native import NativeSampler  # noqa: E402

C = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
wl = bench.workload(2, 0, 1, C)
ns = NativeSampler(wl["ptas"], wl["cfgs"], 0)
ns.alloc(C)
ns.set_state(**wl["init"])
ns.sweep(300, seed=1)
s0 = 300
buf = torch.zeros((C, 20), dtype=torch.int64, device=ns.tdev)
for K in (1, 5, 20, 100, 500):
    buf.zero_()
    _abi.check(ns.lib, ns.lib.gst_debug_stamps(ns.ctx, ct.c_void_p(buf.data_ptr())), "stamps")
    ns.sweep(K, seed=1, sweep0=s0)
    ns.synchronize()
    s0 += K
    ms = ns.last_kernel_ms()
    cyc = buf.cpu().numpy().astype(np.float64)
    tot = cyc[:, :7].sum(axis=1)
    per = tot / K
    # the two chains sharing a SIMD (waves w and w+4 of the CU's two workgroups are not
    # known here; report the chain spread itself)
    print(f"K={K:4d} kernel {ms / K * 1e3:7.1f} us/sweep | per-chain cycles/sweep: mean {per.mean():8.0f} "
          f"p50 {np.median(per):8.0f} p99 {np.percentile(per, 99):8.0f} max {per.max():8.0f} "
          f"max/mean {per.max() / per.mean():.3f} | lnL evals/sweep mean {cyc[:, 16].mean() / K:.2f} "
          f"max {cyc[:, 16].max() / K:.2f}", flush=True)
    _abi.check(ns.lib, ns.lib.gst_debug_stamps(ns.ctx, ct.c_void_p(0)), "stamps off")
