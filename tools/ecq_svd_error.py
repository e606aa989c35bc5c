"""How wrong is the reference's SVD b draw on the ecq posterior?  (cause.)

tools/ecq_theta_bias.py separates the GPU chain from the reference chain into samplers and b
draw; this measures the b draw directly, at the states the reference itself visits.  It runs
the reference algorithm (the oracle with gibbs.py's legacy RNG calls and SVD draw -- bit for
bit the reference's chains, tests/test_oracle_golden.py) and at every sweep after burn-in
compares, for the Sigma = T^T N^-1 T + Phi^-1 and d of that sweep's b draw (gibbs.py:145-182):

* the SVD mean u (u^T d / s) with the exact mean Sigma^-1 d (long double Cholesky), as a
  Mahalanobis distance in units of the conditional's own spread: sqrt(dm^T Sigma dm);
* the SVD draw's square root Li = u s^-1/2 against the exact one: the singular values of
  W = L^T Li (L the long-double Cholesky factor of Sigma), all 1 for an exact draw; a value
  below 1 is a direction in which the reference's draw is narrower than the conditional.

    python tools/ecq_svd_error.py SWEEPS CHAINS [dataset] [burn]
"""
from __future__ import annotations

import json
import os
import sys
import warnings
from multiprocessing import Pool

import numpy as np
import scipy.linalg as sl

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def _chain(args):
    dataset, sweeps, burn, seed = args
    warnings.simplefilter("ignore")
    from golden_io import load_dataset
    from gibbs_student_t_amd.run_sims import MODELS
    from oracle.gibbs_oracle import (LegacyNumpyVariates, Oracle, OutlierModel, _cholesky_ld,
                                     initial_state)
    pta = load_dataset(dataset=dataset)
    np.random.seed(seed)
    x = np.array(pta.sample_params(), dtype=np.float64)
    orc = Oracle(pta, OutlierModel(**MODELS["beta"]))
    st = initial_state(pta, orc.cfg)
    src = LegacyNumpyVariates()
    rows = []
    names = [p.name for p in pta.params]
    for i in range(sweeps):
        if i >= burn:
            # the Sigma, d of this sweep's b draw: the sweep's white + hyper blocks first, on a
            # copy of the RNG stream so the chain itself is the reference's
            rs = np.random.get_state()
            st2 = st.copy()
            orc.cache = None
            xw = orc.white_block(st2, x, src)
            xh = orc.hyper_block(st2, xw, src)
            np.random.set_state(rs)
            Sigma, d = orc.sigma_matrix(st2, xh)
            u, s, _ = sl.svd(Sigma)
            m_svd = u @ ((u.T @ d) / s)
            Li = u * np.sqrt(1 / s)
            L, ok = _cholesky_ld(Sigma)
            if ok:
                ld = np.longdouble
                # exact mean in long double: forward then back substitution
                dd = d.astype(ld)
                zz = np.zeros_like(dd)
                for k in range(len(dd)):
                    zz[k] = (dd[k] - np.dot(L[k, :k], zz[:k])) / L[k, k]
                vv = np.zeros_like(dd)
                for k in range(len(dd) - 1, -1, -1):
                    vv[k] = (zz[k] - np.dot(L[k + 1:, k], vv[k + 1:])) / L[k, k]
                dm = (m_svd.astype(ld) - vv)
                maha = float(np.sqrt(max(float(dm @ (Sigma.astype(ld) @ dm)), 0.0)))
                W = (L.T @ Li.astype(ld)).astype(np.float64)
                sv = np.linalg.svd(W, compute_uv=False)
            else:
                maha, sv = float("nan"), np.array([float("nan")])
            piv = np.diag(np.linalg.cholesky(Sigma[np.ix_(orc.internal_order(),
                                                          orc.internal_order())])) ** 2
            rows.append(dict(sweep=i, cond=float(s[0] / s[-1]), pivot_ratio=float(piv.min() / piv.max()),
                             maha=maha, sv_min=float(sv.min()), sv_max=float(sv.max()),
                             theta=float(st.theta), nu=float(st.nu), zsum=float(np.sum(st.z)),
                             ecorr=[float(v) for nm, v in zip(names, xh) if "ecorr" in nm]))
        x = orc.sweep(st, x, src, b_mean="svd")
    return rows


def main():
    sweeps, chains = int(sys.argv[1]), int(sys.argv[2])
    dataset = sys.argv[3] if len(sys.argv) > 3 else "ecq"
    burn = int(sys.argv[4]) if len(sys.argv) > 4 else 500
    os.environ.setdefault("OPENBLAS_NUM_THREADS", "1")
    with Pool(min(chains, 8)) as pool:
        res = pool.map(_chain, [(dataset, sweeps, burn, 55000 + c) for c in range(chains)])
    rows = [r for rr in res for r in rr]
    maha = np.array([r["maha"] for r in rows])
    svm = np.array([r["sv_min"] for r in rows])
    cond = np.array([r["cond"] for r in rows])
    out = {"dataset": dataset, "states": len(rows), "chains": chains, "sweeps": sweeps,
           "burn": burn,
           "cond_quantiles": {q: float(np.nanquantile(cond, q)) for q in (0.1, 0.5, 0.9, 0.99)},
           "mean_error_sd": {q: float(np.nanquantile(maha, q)) for q in (0.5, 0.9, 0.99)},
           "frac_mean_error_gt_0.1sd": float(np.nanmean(maha > 0.1)),
           "draw_sd_ratio_min": {q: float(np.nanquantile(svm, q)) for q in (0.01, 0.1, 0.5)},
           "frac_draw_narrower_10pct": float(np.nanmean(svm < 0.9))}
    # theta against the b draw's error: the sweeps where the SVD draw is off
    bad = (maha > 0.1) | (svm < 0.9)
    th = np.array([r["theta"] for r in rows])
    out["theta_mean_bad_sweeps"] = float(th[bad].mean()) if bad.any() else None
    out["theta_mean_good_sweeps"] = float(th[~bad].mean()) if (~bad).any() else None
    print(json.dumps(out, indent=1))
    np.save("/tmp/ecq_svd_rows.npy", np.array([[r["cond"], r["pivot_ratio"], r["maha"], r["sv_min"],
                                                 r["theta"], r["zsum"]] for r in rows]))


if __name__ == "__main__":
    main()
