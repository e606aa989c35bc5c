"""Per-chain time of the chains that share a SIMD (diagnostic libgst_stamps.so).

    GST_LIB=gibbs_student_t_amd/libgst_stamps.so python tools/chain_pairs.py [C] [K]
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
K = int(sys.argv[2]) if len(sys.argv) > 2 else 500
wl = bench.workload(2, 0, 1, C)
ns = NativeSampler(wl["ptas"], wl["cfgs"], 0)
ns.alloc(C)
ns.set_state(**wl["init"])
ns.sweep(300, seed=1)
buf = torch.zeros((C, 20), dtype=torch.int64, device=ns.tdev)
_abi.check(ns.lib, ns.lib.gst_debug_stamps(ns.ctx, ct.c_void_p(buf.data_ptr())), "stamps")
ns.sweep(K, seed=1, sweep0=300)
ns.synchronize()
print(f"kernel {ns.last_kernel_ms() / K * 1e3:.1f} us/sweep")
cyc = buf.cpu().numpy().astype(np.float64)
per = cyc[:, :7].sum(axis=1) / K
work = cyc[:, 16] / K
h = C // 2
print(f"chains [0,{h}): mean {per[:h].mean():.0f}  [{h},{C}): mean {per[h:].mean():.0f}")
for a, b in ((0, h), (0, 4)):
    print(f"corr(per[c], per[c+{b}]) = {np.corrcoef(per[:C - b], per[b:])[0, 1]:.3f}" if b else "")
d = per[:h] - per[h:]
print(f"per[c] - per[c+{h}]: mean {d.mean():.0f} sd {d.std():.0f}; frac c faster {np.mean(d < 0):.3f}")
print("deciles of per-chain cycles/sweep:", np.percentile(per, [0, 10, 50, 90, 99, 100]).round(0))
print("corr(per, lnL evals/sweep):", np.corrcoef(per, work)[0, 1].round(3))
for w in range(4):
    print(f"wave slot {w}: mean {per[w::4].mean():.0f}")
