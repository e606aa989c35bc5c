"""Dump every record of a seeded headline run (for bitwise A/B of two library builds):
    GST_LIB=... python tools/diag/lib_records.py out.npz [C] [S]"""
import sys

import numpy as np

sys.path.insert(0, ".")
import bench  # noqa: E402
from gibbs_student_t_amd.native import NativeSampler  # noqa: E402

out = sys.argv[1]
C = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
S = int(sys.argv[3]) if len(sys.argv) > 3 else 60
wl = bench.workload(2, 0, 1, C)
ns = NativeSampler(wl["ptas"], wl["cfgs"], 0)
ns.alloc(C)
ns.set_state(**wl["init"])
rec = ns.alloc_records(S, keys=("x", "b", "z", "alpha", "pout", "theta", "nu"))
ns.sweep(S, records=rec, seed=11, sweep0=0)
np.savez(out, **{k: v.cpu().numpy() for k, v in rec.items()})
