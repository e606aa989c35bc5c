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
import json
import os

import numpy as np
import pytest
import scipy.stats

from golden_io import GOLDEN, load_dataset

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a HIP device", allow_module_level=True)

from gibbs_student_t_amd._abi import STATUS_ERRORS, STATUS_FLOOR  # noqa: E402
from gibbs_student_t_amd.native import NativeSampler  # noqa: E402
from gibbs_student_t_amd.run_sims import MODELS, TRAP_WARN_FRAC  # noqa: E402

P_MIN = 1e-3
# vvh17 starts every chain with all TOAs flagged as outliers (z = 1, gibbs.py:50-51) and a
# fixed alpha = 1e10, so at first every TOA is effectively removed from the fit and Sigma's
# condition number is ~1e22.  The reference's SVD b draw (gibbs.py:169-180) returns the
# smallest eigenvalues at LAPACK's rounding floor, which narrows the timing-model part of the
# draw; that is how its chains leave this all-outlier state within ~100 sweeps (the exact
# draw stays in it for thousands).  The HIP path reproduces the floor (include/gst.h
# gst_sweep: the exact draw from Sigma + f I there, status & 16), so the reference's start
# and burn-in are used unchanged; tests/golden/vvh17_escape_ref.json holds the escape
# sweeps of the reference algorithm itself (the oracle with gibbs.py's legacy RNG and SVD
# draw, tools/vvh17_escape.py) from 256 prior draws.
TRAPPED = 0.5      # all-outlier state: sum z >= n / 2 (run_sims.TRAP_WARN_FRAC's criterion)


def _all_outlier_chains(theta):
    """Chains whose window-mean theta is >= 1/2: the all-outlier state (see above)."""
    return theta.mean(axis=1) >= TRAPPED


@pytest.mark.parametrize("model", ["beta", "t", "gaussian", "uniform", "vvh17"])
def test_posterior_marginals_match_reference(model):
    path = os.path.join(GOLDEN, f"posterior_ref_j1713_{model}.npz")
    ref = np.load(path, allow_pickle=False)
    burn, thin = int(ref["burn"]), 2 * int(ref["thin"])
    rx, rth, rnu = ref["x"][:, ::2], ref["theta"][:, ::2], ref["nu"][:, ::2]
    pta = load_dataset()
    if model == "vvh17":
        # from the reference's all-outlier start a few chains escape only after ~500 sweeps
        # (as the reference's do, test_vvh17_reference_start_escapes_as_the_reference); this
        # 3000-sweep window must start after they have mixed (slow gamma), where the
        # reference's 8 x 40000 draws are dominated by converged sweeps
        burn = 5000
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
    assert np.all((ns.get_state()["status"] & STATUS_ERRORS) == 0)
    if model == "vvh17":
        # the reference's own start and burn-in (1000): chains still in the all-outlier state
        # are unconverged, not posterior samples; both samplers leave it within a few hundred
        # sweeps (test_vvh17_reference_start_escapes_as_the_reference), so they are rare here
        # and are dropped from both samples by the same documented criterion
        trapped = _all_outlier_chains(got["theta"])
        assert trapped.mean() <= 0.01, f"{trapped.sum()} vvh17 chains in the all-outlier state"
        got = {k: v[~trapped] for k, v in got.items()}
        rtrap = _all_outlier_chains(rth)
        assert not rtrap.any()
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


def _vvh17_protocol_run(start, C=1024, seed=31, exact=False, sweeps=10000, chunk=100):
    """vvh17 at the reference study's protocol: 10000 sweeps from prior draws, records
    [100:] (run_sims.py:110-124), from the reference's z = 1 start or run_sims' 'clean'
    z = 0 start; returns the window draws, the all-outlier fraction every `chunk` sweeps and
    each chain's escape sweep (end of the first chunk with sum z < n / 2; -1: never).
    ``exact``: GST_DEBUG_EXACT_BDRAW (no SVD noise floor)."""
    pta = load_dataset()
    n = pta.n
    ns = NativeSampler(pta, MODELS["vvh17"], 0)
    ns.alloc(C)
    ns.set_debug(exact_bdraw=exact)
    lo = np.array([p.pmin for p in pta.params])
    hi = np.array([p.pmax for p in pta.params])
    x0 = np.stack([np.random.default_rng([seed, c]).uniform(lo, hi) for c in range(C)])
    ns.set_state(x=x0, z=np.full((C, n), 1.0 if start == "reference" else 0.0),
                 alpha=np.full((C, n), 1e10), theta=np.full(C, 0.01), nu=np.full(C, 4.0))
    xs, th, frac = [], [], []
    esc = np.full(C, -1)
    for k in range(sweeps // chunk):
        rec = ns.alloc_records(chunk, keys=("x", "theta"))
        ns.sweep(chunk, records=rec, seed=seed, sweep0=chunk * k)
        z = ns.state["z"][:, :n].sum(1).cpu().numpy()
        frac.append(float(np.mean(z >= TRAPPED * n)))
        esc[(esc < 0) & (z < TRAPPED * n)] = chunk * (k + 1)
        xs.append(rec["x"].cpu().numpy())
        th.append(rec["theta"].cpu().numpy())
    status = ns.get_state()["status"]
    assert np.all((status & STATUS_ERRORS) == 0)
    ns.close()
    return np.concatenate(xs, 1)[:, 100:], np.concatenate(th, 1)[:, 100:], frac, esc, status


def escape_vs_reference(esc, trapped_at):
    """KS p of the GPU's escape sweeps (10-sweep bins, -1: not escaped) against the reference
    algorithm's (tests/golden/vvh17_escape_ref.json, binned alike), and Fisher-exact p of the
    trapped counts at each sweep in ``trapped_at``."""
    with open(os.path.join(GOLDEN, "vvh17_escape_ref.json")) as f:
        ref = json.load(f)
    big = 10 ** 6
    r = np.array([e if e is not None else big for e in ref["escape"]], float)
    r = 10 * np.ceil(r / 10)
    g = np.where(esc > 0, esc, big).astype(float)
    ks = scipy.stats.ks_2samp(g, r).pvalue
    fisher = {}
    for s_ in trapped_at:
        a, b = int(np.sum(g > s_)), int(np.sum(r > s_))
        fisher[s_] = (a / len(g), b / len(r),
                      scipy.stats.fisher_exact([[a, len(g) - a], [b, len(r) - b]])[1])
    return ks, fisher, float(np.median(g)), float(np.median(r))


def test_vvh17_reference_start_escapes_as_the_reference():
    """The reference's own z = 1 start: the chains leave the all-outlier state as the
    reference algorithm's do -- escape sweeps against the oracle with gibbs.py's SVD draw
    (256 prior draws, binned to the 10-sweep resolution of this run): KS p > 1e-3, trapped
    fractions at sweeps 200 / 500 / 1000 consistent with the reference's (Fisher p > 1e-3)
    and at most 1% at sweep 500; every chain drew at the SVD noise floor at its start."""
    _, _, frac, esc, status = _vvh17_protocol_run("reference", sweeps=1000, chunk=10)
    ks, fisher, gmed, rmed = escape_vs_reference(esc, (200, 500, 1000))
    print(f"\nvvh17 escape: gpu median {gmed} reference median {rmed} KS p {ks:.3g}; "
          f"trapped (gpu, reference, Fisher p): {fisher}")
    assert np.all(status & STATUS_FLOOR)
    assert frac[49] <= 0.01, f"trapped at sweep 500: {frac[49]:.3f}"
    assert ks > P_MIN, f"escape sweeps: KS p={ks:.2e} (gpu median {gmed}, reference {rmed})"
    for s_, (a, b, p) in fisher.items():
        assert p > P_MIN, f"trapped at sweep {s_}: gpu {a:.4f} reference {b:.4f} p={p:.2e}"


def test_vvh17_reference_protocol_reference_start_matches_reference():
    """run_sims' default vvh17 start -- the reference's z = 1 -- at the reference's own
    protocol (10000 sweeps, records [100:]): the window's marginals pass KS against the
    reference's posterior draws WITHOUT dropping any chain (the few chains that leave the
    all-outlier state late contribute a negligible share of the 9900-record window)."""
    ref = np.load(os.path.join(GOLDEN, "posterior_ref_j1713_vvh17.npz"), allow_pickle=False)
    thin = 2 * int(ref["thin"])
    x, th, frac, _, _ = _vvh17_protocol_run("reference")
    assert max(frac[5:]) <= 0.01          # at most 1% in the all-outlier state after 600
    names = [str(s) for s in ref["names"]]
    for j, nm in enumerate(names):
        p = scipy.stats.ks_2samp(x[:, ::thin, j].ravel(), ref["x"][:, ::2, j].ravel()).pvalue
        assert p > P_MIN, f"vvh17 reference start {nm}: KS p={p:.2e}"
    p = scipy.stats.ks_2samp(th[:, ::thin].ravel(), ref["theta"][:, ::2].ravel()).pvalue
    assert p > P_MIN, f"vvh17 reference start theta: KS p={p:.2e}"


def test_vvh17_reference_protocol_clean_start_matches_reference():
    """run_sims' optional clean vvh17 start (z = 0) at the reference's own protocol: no chain
    ever in the all-outlier state and the [100:] window's marginals pass KS against the
    reference's posterior draws WITHOUT dropping any chain."""
    ref = np.load(os.path.join(GOLDEN, "posterior_ref_j1713_vvh17.npz"), allow_pickle=False)
    thin = 2 * int(ref["thin"])
    x, th, frac, _, _ = _vvh17_protocol_run("clean")
    assert max(frac) == 0.0
    names = [str(s) for s in ref["names"]]
    for j, nm in enumerate(names):
        p = scipy.stats.ks_2samp(x[:, ::thin, j].ravel(), ref["x"][:, ::2, j].ravel()).pvalue
        assert p > P_MIN, f"vvh17 clean start {nm}: KS p={p:.2e}"
    p = scipy.stats.ks_2samp(th[:, ::thin].ravel(), ref["theta"][:, ::2].ravel()).pvalue
    assert p > P_MIN, f"vvh17 clean start theta: KS p={p:.2e}"


def test_vvh17_exact_draw_trap_is_the_documented_one():
    """The reference's z = 1 start with the EXACT b draw (GST_DEBUG_EXACT_BDRAW: no SVD noise
    floor), at the reference's protocol: the all-outlier fraction follows the envelope
    measured in round 3 (every chain trapped through sweep 200, most through 500, nearly
    none by 10000) -- the behaviour the floor removes."""
    _, th, frac, _, status = _vvh17_protocol_run("reference", exact=True)
    assert not np.any(status & STATUS_FLOOR)
    assert frac[1] >= 0.95           # sweep 200
    assert frac[4] >= 0.5            # sweep 500
    assert frac[-1] <= 0.02          # sweep 10000
    assert np.mean(th >= 0.5) > TRAP_WARN_FRAC      # run_sims would flag this entry
