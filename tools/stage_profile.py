"""Per-stage cycle breakdown of the sweep kernel (diagnostic libgst_stamps.so).

Usage: GST_LIB=gibbs_student_t_amd/libgst_stamps.so python tools/stage_profile.py [C] [S] [waves]
(SP_CONFIG=3: bench config 3's pulsar instead of J1713+0747)
Stamps fence the overlaps of the real kernel: read the SHARES, not the absolute length.
"""
import ctypes as ct
import os
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from gibbs_student_t_amd import _abi, data  # noqa: E402
from gibbs_student_t_amd.model import PTA  # noqa: E402
from gibbs_student_t_amd.native import NativeSampler  # noqa: E402

STAGES = ["record", "white MH", "Gram+TM elim", "hyper MH (11 chol)", "b draw",
          "theta+z+alpha", "nu", "(hyper: phi + S0 load)", "(hyper: F elimination)",
          "(gram: MFMA loop)", "(gram: transpose+prior)", "(gram: TM chol)",
          "(b: yinv + rhs)", "(b: back-subst)", "(b: T b)", "(white: lnL evals)"]


def main():
    C = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    S = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    waves = int(sys.argv[3]) if len(sys.argv) > 3 else "auto"
    if os.environ.get("SP_CONFIG") == "3":   # bench config 3's pulsar (130 distinct sigmas)
        import bench
        wl = bench.workload(3, 0, 1, C)
        ns = NativeSampler(wl["ptas"], wl["cfgs"], 0)
        ns.set_waves(waves)
        ns.alloc(C)
        ns.set_state(**wl["init"])
    else:
        pta = PTA(data.j1713())
        ns = NativeSampler(pta, dict(model="mixture", vary_df=True, theta_prior="beta"), 0)
        ns.set_waves(waves)
        ns.alloc(C)
        rng = np.random.default_rng(0)
        x0 = np.stack([[rng.uniform(1, 7), rng.uniform(-18, -12), rng.uniform(-10, -5)]
                       for _ in range(C)])
        ns.set_state(x=x0, z=np.ones((C, ns.n)), alpha=np.ones((C, ns.n)),
                     theta=np.full(C, 0.01), nu=np.full(C, 4.0))
    ns.sweep(300, seed=1)
    buf = torch.zeros((C, 28), dtype=torch.int64, device=ns.tdev)
    _abi.check(ns.lib, ns.lib.gst_debug_stamps(ns.ctx, ct.c_void_p(buf.data_ptr())),
               "gst_debug_stamps")
    ns.sweep(S, seed=1, sweep0=300)
    ns.synchronize()
    ms = ns.last_kernel_ms()
    cyc = buf.cpu().numpy().astype(np.float64) / S
    tot = cyc[:, :7].sum(axis=1)
    print(f"C={C} S={S} waves={waves} kernel {ms:.2f} ms = {ms / S * 1e3:.1f} us/sweep; "
          f"stamped cycles/sweep/chain median {np.median(tot):.0f}")
    for i, nm in enumerate(STAGES):
        print(f"  {nm:22s} {np.median(cyc[:, i]):10.0f} cyc  {np.median(cyc[:, i] / tot) * 100:5.1f} %")

    for i, nm in ((19, "(hyper: harvest + stats)"), (20, "(record: MH variates)"),
                  (21, "(white: class sums)"), (22, "(white: lane lnL tree)"),
                  (23, "(outlier: theta)"), (24, "(outlier: z)"), (25, "(outlier: alpha)")):
        print(f"  {nm:22s} {np.median(cyc[:, i]):10.0f} cyc  "
              f"{np.median(cyc[:, i] / tot) * 100:5.1f} %")
    for i, nm in ((16, "red-noise lnL evaluations"), (17, "two-wave rounds"),
                  (18, "accepted red-noise proposals")):
        print(f"  {nm:30s} {cyc[:, i].mean():6.2f} per sweep")


if __name__ == "__main__":
    main()
