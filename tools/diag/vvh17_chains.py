"""Diagnostic: per-chain posterior summaries of the vvh17 model on the golden J1713 data."""
import sys
import numpy as np
sys.path.insert(0, "."); sys.path.insert(0, "tests")
from golden_io import load_dataset
from gibbs_student_t_amd.native import NativeSampler
from gibbs_student_t_amd.run_sims import MODELS

model = sys.argv[1] if len(sys.argv) > 1 else "vvh17"
pta = load_dataset()
C, S = 1024, 3000
burn = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
cfg = MODELS[model]
ns = NativeSampler(pta, cfg, 0)
ns.alloc(C)
lo = np.array([p.pmin for p in pta.params]); hi = np.array([p.pmax for p in pta.params])
x0 = np.random.default_rng(5).uniform(lo, hi, size=(C, len(lo)))
a0 = 1.0 if cfg.get("vary_alpha", True) else float(cfg["alpha"])
ns.set_state(x=x0, z=np.full((C, pta.n), 1.0), alpha=np.full((C, pta.n), a0),
             theta=np.full(C, 0.01), nu=np.full(C, 4.0))
ns.sweep(burn, seed=77)
rec = ns.alloc_records(S, keys=("x", "z", "theta"))
ns.sweep(S, records=rec, seed=77, sweep0=burn)
x = rec["x"].cpu().numpy(); z = rec["z"].cpu().numpy(); th = rec["theta"].cpu().numpy()
gm = x[:, :, 0].mean(1); zs = z.sum(2).mean(1)
print("status", np.unique(ns.get_state()["status"], return_counts=True))
print("gamma chain-mean quantiles", np.quantile(gm, [0, .05, .25, .5, .75, .95, 1]).round(2))
print("logA quantiles", np.quantile(x[:, :, 1].mean(1), [0, .05, .5, .95, 1]).round(2))
print("equad quantiles", np.quantile(x[:, :, 2].mean(1), [0, .05, .5, .95, 1]).round(2))
print("sum z per chain quantiles", np.quantile(zs, [0, .05, .25, .5, .75, .95, 1]).round(2))
print("theta mean", th.mean(), "overall gamma mean", x[:, :, 0].mean())
for lo_, hi_ in ((0, 2), (2, 5), (5, 200)):
    sel = (zs >= lo_) & (zs < hi_)
    if sel.any():
        print(f"chains with {lo_}<=sum z<{hi_}: {sel.sum()}, gamma mean {gm[sel].mean():.3f}")
