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
from gibbs_student_t_amd.run_sims import MODELS, TRAP_WARN_FRAC  # noqa: E402

P_MIN = 1e-3
# vvh17 starts every chain with all TOAs flagged as outliers (z = 1, gibbs.py:50-51) and a
# fixed alpha = 1e10, so at first every TOA is effectively removed from the fit, b is drawn
# from its prior, and q ~ 1 keeps z = 1: a metastable all-outlier state that an exact b draw
# leaves only slowly.  The reference's chains leave it within ~200 sweeps only through its SVD
# square root of a Sigma with cond ~ 1e22 (tests/golden/ref_vvh17_*.npz): the oracle with the
# reference's SVD draw escapes in 100-200 sweeps, the same oracle with only the b draw made
# exact (Cholesky) stays trapped for 900-1500+ (tools/diag/vvh17_trap_cpu.py).  Measured on
# the GPU at the reference's study protocol (tools/vvh17_protocol.py, profiles/
# r3_vvh17_protocol.json): 100% of 1024 chains trapped at sweep 500, 78% at 1000, 25% at
# 2000, 1.5% at 5000, 0.3% at 10000.  So this comparison burns in longer, and drops the
# chains whose window still sits in that state by the documented criterion
# (run_sims.TRAP_WARN_FRAC: sum z >= n/2, i.e. theta >= 1/2 for vvh17's uniform theta
# prior, theta ~ Beta(sum z + 1, n - sum z + 1)), applied to BOTH samples' chains.
VVH17_BURN = 30000


def _all_outlier_chains(theta):
    """Chains whose window-mean theta is >= 1/2: the all-outlier state (see above)."""
    return theta.mean(axis=1) >= 0.5


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
        # the same documented criterion on both samples: chains still in the all-outlier
        # state are unconverged, not samples of the posterior; they must be rare here, and
        # the reference's chains (burn-in 1000, escaped through the SVD draw) have none
        trapped = _all_outlier_chains(got["theta"])
        assert trapped.mean() <= 0.01, f"{trapped.sum()} vvh17 chains in the all-outlier state"
        got = {k: v[~trapped] for k, v in got.items()}
        rtrap = _all_outlier_chains(rth)
        assert not rtrap.any()
        rx, rth, rnu = rx[~rtrap], rth[~rtrap], rnu[~rtrap]
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


def _vvh17_protocol_run(start, C=1024, seed=31):
    """vvh17 at the reference study's protocol: 10000 sweeps from prior draws, records
    [100:] (run_sims.py:110-124), from the reference's z = 1 start or run_sims' 'clean'
    z = 0 start; returns the window draws and the all-outlier fraction every 100 sweeps."""
    pta = load_dataset()
    n = pta.n
    ns = NativeSampler(pta, MODELS["vvh17"], 0)
    ns.alloc(C)
    lo = np.array([p.pmin for p in pta.params])
    hi = np.array([p.pmax for p in pta.params])
    x0 = np.stack([np.random.default_rng([seed, c]).uniform(lo, hi) for c in range(C)])
    ns.set_state(x=x0, z=np.full((C, n), 1.0 if start == "reference" else 0.0),
                 alpha=np.full((C, n), 1e10), theta=np.full(C, 0.01), nu=np.full(C, 4.0))
    xs, th, frac = [], [], []
    for k in range(100):
        rec = ns.alloc_records(100, keys=("x", "theta"))
        ns.sweep(100, records=rec, seed=seed, sweep0=100 * k)
        z = ns.state["z"][:, :n].sum(1)
        frac.append(float((z >= 0.5 * n).double().mean()))
        xs.append(rec["x"].cpu().numpy())
        th.append(rec["theta"].cpu().numpy())
    assert np.all(ns.get_state()["status"] == 0)
    ns.close()
    return np.concatenate(xs, 1)[:, 100:], np.concatenate(th, 1)[:, 100:], frac


def test_vvh17_reference_protocol_clean_start_matches_reference():
    """run_sims' default vvh17 start (z = 0) at the reference's own protocol: no chain ever
    in the all-outlier state and the [100:] window's marginals pass KS against the
    reference's posterior draws WITHOUT dropping any chain."""
    ref = np.load(os.path.join(GOLDEN, "posterior_ref_j1713_vvh17.npz"), allow_pickle=False)
    thin = 2 * int(ref["thin"])
    x, th, frac = _vvh17_protocol_run("clean")
    assert max(frac) == 0.0
    names = [str(s) for s in ref["names"]]
    for j, nm in enumerate(names):
        p = scipy.stats.ks_2samp(x[:, ::thin, j].ravel(), ref["x"][:, ::2, j].ravel()).pvalue
        assert p > P_MIN, f"vvh17 clean start {nm}: KS p={p:.2e}"
    p = scipy.stats.ks_2samp(th[:, ::thin].ravel(), ref["theta"][:, ::2].ravel()).pvalue
    assert p > P_MIN, f"vvh17 clean start theta: KS p={p:.2e}"


def test_vvh17_reference_start_trap_is_the_documented_one():
    """The reference's z = 1 start with the exact b draw, at the reference's protocol: the
    all-outlier fraction follows the measured envelope documented in DESIGN.md section 3
    (every chain trapped through sweep 200, most through 500, nearly none by 10000) --
    a known behavioural difference from gibbs.py's SVD draw, flagged by run_sims."""
    _, th, frac = _vvh17_protocol_run("reference")
    assert frac[1] >= 0.95           # sweep 200
    assert frac[4] >= 0.5            # sweep 500
    assert frac[-1] <= 0.02          # sweep 10000
    assert np.mean(th >= 0.5) > TRAP_WARN_FRAC      # run_sims would flag this entry
