"""The on-device batched generator (gst_simulate, csrc/gst_sim.hpp) against its CPU
restatement oracle/sim_oracle.py (same Philox stream), the simulate_data.py:10-39 recipe.

Exact: the outlier flags (a uniform compared with theta).  Close: error bars (pow on device
vs numpy, <= 1e-14 relative), residuals and the clean twin (summation order of F coef and
the refit; <= 1e-12 of the residual scale)."""
import numpy as np
import pytest

from gibbs_student_t_amd import data
from gibbs_student_t_amd.model import FYR, fourier_basis, svd_tm_basis
from gibbs_student_t_amd.simulate import pairs, simulate_batch
from oracle import sim_oracle as so

pytestmark = pytest.mark.gpu


def _j1713():
    raw = data.load_j1713_raw()
    mjd = raw["mjd_int"].astype(np.float64) + raw["mjd_frac"]
    return mjd * data.DAY_SEC, data.design_matrix(mjd, raw["par"], raw["fit"]), raw


def _oracle(toas, M, d, **kw):
    U = svd_tm_basis(M)[0]
    F, ff = fourier_basis(toas, 30)
    f = ff[::2]
    df = np.diff(np.concatenate(([0.0], f)))
    return so.simulate(F, U, dataset=d, lf=np.log(ff), ldf=np.log(np.repeat(df, 2)),
                       log_fyr=np.log(FYR), **kw)


def _check(dev, d, want, scale):
    r, err, z, r2 = want
    np.testing.assert_array_equal(dev["z"][d], z)
    np.testing.assert_allclose(dev["toaerrs"][d], err, rtol=1e-14, atol=0)
    np.testing.assert_allclose(dev["residuals"][d], r, rtol=0, atol=1e-12 * scale)
    if r2 is not None:
        np.testing.assert_allclose(dev["residuals_clean"][d], r2, rtol=0, atol=1e-12 * scale)


def test_powerlaw_lognormal_gaussian():
    """Config-3/4 recipe at the J1713 epochs: log-normal errors, power-law red noise,
    per-dataset theta (the run_sims grid) and red-noise parameters."""
    toas, M, _ = _j1713()
    D = 12
    thetas = np.array([0.05, 0.1, 0.15] * 4)
    lA = np.linspace(-14.5, -13.5, D)
    gam = np.linspace(3.0, 5.0, D)
    dev = simulate_batch(toas, M, D, seed=99, theta=thetas, log10_A=lA, gamma=gam)
    for d in range(D):
        want = _oracle(toas, M, d, seed=99, theta=thetas[d], sigma_out=1e-6,
                       log10_A=lA[d], gamma=gam[d])
        _check(dev, d, want, np.abs(want[0]).max())
    assert 0.02 < dev["z"].mean() < 0.2


def test_red_txt_student_t():
    """Config 3's red.txt realisation and config 4's Student-t white noise (dof = 4)."""
    toas, M, raw = _j1713()
    red = raw["red"] * data.DAY_SEC
    D = 4
    dev = simulate_batch(toas, M, D, seed=7, dataset0=100, theta=0.05, dof=4.0, red=red)
    for d in range(D):
        want = _oracle(toas, M, 100 + d, seed=7, theta=0.05, sigma_out=1e-6, dof=4.0, red=red)
        _check(dev, d, want, np.abs(want[0]).max())


def test_shards_draw_the_same_datasets():
    """dataset0 keys the stream: datasets [4, 8) drawn alone equal that slice of [0, 8)."""
    toas, M, _ = _j1713()
    full = simulate_batch(toas, M, 8, seed=5, theta=0.1)
    part = simulate_batch(toas, M, 4, seed=5, theta=0.1, dataset0=4)
    for k in ("residuals", "toaerrs", "z", "residuals_clean"):
        np.testing.assert_array_equal(full[k][4:], part[k])


def test_large_batch_and_pairs_feed_the_sampler():
    """256 datasets (config 4's grid size) in one launch; the pairs run through the
    sampler's model setup and a few sweeps with finite state."""
    from gibbs_student_t_amd.model import PTA
    from gibbs_student_t_amd.native import NativeSampler
    toas, M, raw = _j1713()
    sim = simulate_batch(toas, M, 256, seed=1, theta=np.repeat([0.05, 0.1, 0.15, 0.2], 64))
    assert sim["residuals"].shape == (256, len(toas))
    assert np.all(np.isfinite(sim["residuals"])) and np.all(np.isfinite(sim["residuals_clean"]))
    pr = pairs(toas, M, sim, name="J1713+0747", freqs=raw["freq_mhz"])
    ptas = [PTA(a) for a, _ in pr[:2]] + [PTA(b) for _, b in pr[:2]]
    cfg = dict(model="mixture", vary_df=True, theta_prior="beta")
    ns = NativeSampler(ptas, cfg, 0)
    C = 64
    ns.alloc(C, dataset=np.repeat(np.arange(4), C // 4))
    lo = np.array([p.pmin for p in ptas[0].params])
    hi = np.array([p.pmax for p in ptas[0].params])
    ns.set_state(x=np.random.default_rng(0).uniform(lo, hi, size=(C, len(lo))),
                 theta=np.full(C, 0.05), nu=np.full(C, 4.0))
    ns.sweep(10, seed=3)
    st = ns.get_state()
    ns.close()
    assert np.all(np.isfinite(st["x"])) and np.all(np.isfinite(st["b"]))
