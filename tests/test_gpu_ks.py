"""Second parity layer: full-run posteriors agree with the reference by KS tests.

tests/golden/posterior_ref_j1713_{model}.npz (all five run_sims.py:89-107 models) holds
thinned draws of the REFERENCE sampler
(gibbs.py, run by tools/gen_posterior.py in the build container: 8 chains x 40000 sweeps,
burn-in 1000, thinned by 25) on the golden J1713+0747 dataset.  The GPU runs 1024 chains
with on-device Philox variates from prior draws, thinned the same way; every sampled
parameter, theta and the dof nu must pass a two-sample KS test at p > 1e-3 (thinning by 25
sweeps; the test keeps every second of those draws on both sides, i.e. 50 sweeps apart,
beyond the integrated autocorrelation time of every marginal (about 40 sweeps for gamma,
bench.py ESS), so the draws are close to independent as the KS test assumes).
"""
import os

import numpy as np
import pytest
import scipy.stats

from golden_io import GOLDEN, load_dataset

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a HIP device", allow_module_level=True)

from gibbs_student_t_amd.native import NativeSampler  # noqa: E402
from gibbs_student_t_amd.run_sims import MODELS  # noqa: E402

P_MIN = 1e-3
# vvh17 starts every chain with all TOAs flagged as outliers (z = 1, gibbs.py:50-51) and a
# fixed alpha = 1e10, so at first every TOA is effectively removed from the fit, b is drawn
# from its prior, and q ~ 1 keeps z = 1: a metastable state with negligible posterior mass
# that an exact b draw leaves only slowly (measured: after 1000 sweeps most of 1024 chains
# still carry 10-130 outliers; after 20000, all but ~1 in 1000 are at the posterior's ~8).
# The reference's chains leave it within ~200 sweeps only through its SVD square root of a
# Sigma with cond ~ 1e22 (tests/golden/ref_vvh17_*.npz): the oracle with the reference's
# SVD draw escapes in 100-200 sweeps, the same oracle with only the b draw made exact
# (Cholesky) stays trapped for 900-1500+ (tools/diag/vvh17_trap_cpu.py, 4 seeds each).  So
# the vvh17 comparison burns in longer.
VVH17_BURN = 30000


@pytest.mark.parametrize("model", ["beta", "t", "gaussian", "uniform", "vvh17"])
def test_posterior_marginals_match_reference(model):
    path = os.path.join(GOLDEN, f"posterior_ref_j1713_{model}.npz")
    ref = np.load(path, allow_pickle=False)
    burn, thin = int(ref["burn"]), 2 * int(ref["thin"])
    rx, rth, rnu = ref["x"][:, ::2], ref["theta"][:, ::2], ref["nu"][:, ::2]
    pta = load_dataset()
    if model == "vvh17":
        burn = VVH17_BURN
    C, S = 1024, burn + 60 * thin
    ns = NativeSampler(pta, MODELS[model], 0)
    ns.alloc(C)
    lo = np.array([p.pmin for p in pta.params])
    hi = np.array([p.pmax for p in pta.params])
    x0 = np.random.default_rng(5).uniform(lo, hi, size=(C, len(lo)))
    cfg = MODELS[model]
    a0 = 1.0 if cfg.get("vary_alpha", True) else float(cfg["alpha"])   # gibbs.py:44-47
    ns.set_state(x=x0, z=np.full((C, pta.n), 1.0 if cfg["model"] != "gaussian" else 0.0),
                 alpha=np.full((C, pta.n), a0), theta=np.full(C, 0.01), nu=np.full(C, 4.0))
    ns.sweep(burn, seed=77)
    rec = ns.alloc_records(S - burn, keys=("x", "theta", "nu"))
    ns.sweep(S - burn, records=rec, seed=77, sweep0=burn)
    got = {k: v.cpu().numpy()[:, ::thin] for k, v in rec.items()}
    assert np.all(ns.get_state()["status"] == 0)
    if model == "vvh17":
        # chains still caught in the all-outlier state the z = 1 start puts them in (see the
        # module docstring) are unconverged, not samples of the posterior: drop them, and
        # require that they are rare
        tm = got["theta"].mean(axis=1)
        keep = tm < 3 * np.median(tm)
        assert keep.mean() >= 0.99, f"{(~keep).sum()} vvh17 chains unconverged"
        got = {k: v[keep] for k, v in got.items()}
    names = [str(s) for s in ref["names"]]
    series = [(nm, got["x"][..., j].ravel(), rx[..., j].ravel())
              for j, nm in enumerate(names)]
    if MODELS[model]["model"] in ("mixture", "vvh17"):
        series.append(("theta", got["theta"].ravel(), rth.ravel()))
    if MODELS[model].get("vary_df", True):
        series.append(("nu", got["nu"].ravel(), rnu.ravel()))
    for nm, g, r in series:
        res = scipy.stats.ks_2samp(g, r)
        assert res.pvalue > P_MIN, f"{model} {nm}: KS D={res.statistic:.4f} p={res.pvalue:.2e} " \
                                   f"(gpu mean {g.mean():.4g}, ref mean {r.mean():.4g})"
    ns.close()
