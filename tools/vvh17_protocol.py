"""vvh17 at the reference's study protocol, on the GPU.

    python tools/vvh17_protocol.py [chains] [out.json]

run_sims.py runs every model for niter = 10000 sweeps from a prior draw (run_sims.py:
110-113) and keeps records [100:] (:118-124).  vvh17 starts with every TOA flagged
(z = 1) and alpha fixed at 1e10 (gibbs.py:44-51): every TOA is effectively removed, so b
is drawn from its prior and q ~ 1 keeps z = 1.  This measures, for the golden J1713+0747
dataset (the KS fixture's), the fraction of chains still in that all-outlier state
(sum z >= n/2, run_sims.TRAP_WARN_FRAC) every 100 sweeps, and the KS p-values of the
[100:] window against the reference's own posterior draws
(tests/golden/posterior_ref_j1713_vvh17.npz) without dropping any chain -- for the
reference's start and for run_sims' ``vvh17_start='clean'`` (z = 0).
"""
import json
import os
import sys

import numpy as np
import scipy.stats

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "tests"))
from golden_io import GOLDEN, load_dataset  # noqa: E402
from gibbs_student_t_amd.native import NativeSampler  # noqa: E402
from gibbs_student_t_amd.run_sims import MODELS  # noqa: E402

NITER, BURN, CHUNK = 10000, 100, 100


def run(start, C, seed=31):
    pta = load_dataset()
    n = pta.n
    ns = NativeSampler(pta, MODELS["vvh17"], 0)
    ns.alloc(C)
    lo = np.array([p.pmin for p in pta.params])
    hi = np.array([p.pmax for p in pta.params])
    x0 = np.stack([np.random.default_rng([seed, c]).uniform(lo, hi) for c in range(C)])
    ns.set_state(x=x0, z=np.full((C, n), 1.0 if start == "reference" else 0.0),
                 alpha=np.full((C, n), 1e10), theta=np.full(C, 0.01), nu=np.full(C, 4.0))
    curve, xs, th = [], [], []
    for k in range(NITER // CHUNK):
        rec = ns.alloc_records(CHUNK, keys=("x", "theta"))
        ns.sweep(CHUNK, records=rec, seed=seed, sweep0=k * CHUNK)
        z = ns.state["z"][:, :n].sum(1).cpu().numpy()
        curve.append(float(np.mean(z >= 0.5 * n)))
        xs.append(rec["x"].cpu().numpy())
        th.append(rec["theta"].cpu().numpy())
    status = ns.get_state()["status"]
    ns.close()
    x = np.concatenate(xs, axis=1)[:, BURN:]
    theta = np.concatenate(th, axis=1)[:, BURN:]
    return pta, curve, x, theta, int((status != 0).sum())


def ks(pta, x, theta):
    ref = np.load(os.path.join(GOLDEN, "posterior_ref_j1713_vvh17.npz"), allow_pickle=False)
    thin = 2 * int(ref["thin"])
    names = [str(s) for s in ref["names"]]
    out = {}
    for j, nm in enumerate(names):
        r = scipy.stats.ks_2samp(x[:, ::thin, j].ravel(), ref["x"][:, ::2, j].ravel())
        out[nm] = float(r.pvalue)
    r = scipy.stats.ks_2samp(theta[:, ::thin].ravel(), ref["theta"][:, ::2].ravel())
    out["theta"] = float(r.pvalue)
    return out


def main():
    C = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    dst = sys.argv[2] if len(sys.argv) > 2 else None
    res = {"protocol": f"{NITER} sweeps from prior draws, records [{BURN}:] (run_sims.py:"
                       "110-124); golden J1713+0747 dataset, vvh17 model (run_sims.py:89-92)",
           "chains": C, "criterion": "sum z >= n/2 (all-outlier state)"}
    for start in ("reference", "clean"):
        pta, curve, x, theta, nstat = run(start, C)
        chain_trapped_window = float(np.mean(theta.mean(axis=1) >= 0.5))
        res[start] = {"trapped_frac_every_100_sweeps": curve,
                      "trapped_frac_at": {str(s): curve[s // CHUNK - 1]
                                          for s in (100, 200, 500, 1000, 2000, 5000, 10000)},
                      "record_frac_trapped_in_window": float(np.mean(theta >= 0.5)),
                      "chains_with_window_mean_theta_ge_half": chain_trapped_window,
                      "ks_pvalues_no_filter": ks(pta, x, theta),
                      "chains_with_status": nstat}
        print(start, json.dumps(res[start]["trapped_frac_at"]),
              json.dumps(res[start]["ks_pvalues_no_filter"]), flush=True)
    if dst:
        with open(dst, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
