"""Datasets for the sampler: J1713+0747 epochs and the simulate_data.py recipe, batched.

No tempo2 / libstempo / enterprise exist offline, so the pieces the reference gets from
them are restated here and documented as *parity-unpinned* against those tools:

* TOAs, errors, frequencies and fitted-parameter values come from the reference's own
  J1713+0747.tim / .par (packed into ``data/J1713+0747.npz`` by tools/make_j1713_npz.py).
* The timing-model design matrix is an analytic approximation of tempo2's for the fitted
  parameters (J1713+0747.par flag ``1``: RAJ DECJ F0 F1 PMRA PMDEC PX SINI PB T0 A1 OM ECC)
  plus the offset column: 14 columns, as SURVEY.md section 0 counts.  Only the column *span*
  matters to the sampler: the timing model is marginalised with a 1e40 prior on the SVD
  basis (run_sims.py:22-29).
* Residuals are simulated at the real epochs following simulate_data.py:10-39: white noise,
  power-law red noise (A=1e-14, gamma=4.33, 30 components, simulate_data.py:21), Bernoulli(theta)
  outliers with sigma_out = 1e-6 s (simulate_data.py:24-26), then the timing model is fitted
  out (projected away) as tempo2's refit would.
"""
from __future__ import annotations

import os

import numpy as np

from .model import DAY_SEC, FYR, PulsarData, fourier_basis, powerlaw

_HERE = os.path.dirname(os.path.abspath(__file__))
J1713_NPZ = os.path.join(_HERE, "data", "J1713+0747.npz")


def load_j1713_raw():
    """The packed J1713+0747 epochs and par values (see tools/make_j1713_npz.py)."""
    d = np.load(J1713_NPZ, allow_pickle=False)
    par = {str(k): float(v) for k, v in zip(d["par_names"], d["par_values"])}
    fit = [str(k) for k, f in zip(d["par_names"], d["par_fit"]) if f]
    return {
        "mjd_int": d["mjd_int"], "mjd_frac": d["mjd_frac"],
        "toaerr_us": d["toaerr_us"], "freq_mhz": d["freq_mhz"],
        "par": par, "fit": fit, "red": d["red"],
    }


def design_matrix(mjd: np.ndarray, par: dict, fit: list) -> np.ndarray:
    """Approximate tempo2 design matrix: offset + one column per fitted parameter.

    Each column is the leading-order derivative of the timing residual w.r.t. that
    parameter (spin: polynomial in t; astrometry: annual / semi-annual terms; DD binary:
    Roemer-delay derivatives in orbital phase plus the Shapiro-delay SINI term).
    """
    pep = par.get("PEPOCH", 53000.0)
    t = (mjd - pep) * DAY_SEC
    lam = 2.0 * np.pi * (mjd - 51544.5) / 365.25 - np.deg2rad(par.get("RAJ", 0.0))
    pb = par.get("PB", 1.0)
    t0 = par.get("T0", pep)
    a1 = par.get("A1", 1.0)
    om = np.deg2rad(par.get("OM", 0.0))
    ecc = par.get("ECC", 0.0)
    sini = par.get("SINI", 0.0)
    r_sh = 4.925490947e-6 * par.get("M2", 0.0)
    phase = 2.0 * np.pi * (mjd - t0) / pb
    cols = {
        "F0": t / DAY_SEC, "F1": 0.5 * (t / DAY_SEC) ** 2,
        "RAJ": np.cos(lam), "DECJ": np.sin(lam),
        "PMRA": (t / DAY_SEC) * np.cos(lam), "PMDEC": (t / DAY_SEC) * np.sin(lam),
        "PX": np.cos(2.0 * lam),
        "A1": np.sin(phase + om) + 0.5 * ecc * np.sin(2 * phase + om),
        "OM": a1 * (np.cos(phase + om) + 0.5 * ecc * np.cos(2 * phase + om)
                    - 1.5 * ecc * np.cos(om)),
        "T0": -(2 * np.pi / pb) * a1 * (np.cos(phase + om) + ecc * np.cos(2 * phase + om)),
        "PB": -(2 * np.pi * (mjd - t0) / pb ** 2) * a1 * np.cos(phase + om),
        "ECC": a1 * (0.5 * np.sin(2 * phase + om) - 1.5 * np.sin(om)
                     + 0.25 * np.sin(3 * phase + om)),
        "SINI": 2 * r_sh * np.sin(phase + om) / (1.0 - sini * np.sin(phase + om)),
    }
    M = [np.ones_like(mjd)]
    for name in fit:
        if name in cols:
            M.append(cols[name])
    return np.column_stack(M)


def simulate_residuals(toas, toaerrs, U, *, theta=0.05, sigma_out=1e-6, log10_A=-14.0,
                       gamma=4.33, components=30, rng=None, red=None, dof=None):
    """One realisation of the simulate_data.py:10-39 recipe at given epochs.

    Returns ``(residuals, z)``: white + red + outliers with the timing model projected
    out (``r - U U^T r``); ``z`` are the injected outlier flags.  ``dof`` (not in the
    reference; the BASELINE config-4 Student-t grid) replaces the Gaussian white noise of
    the non-outlier TOAs by sigma * t_dof draws.
    """
    rng = np.random.default_rng() if rng is None else rng
    n = len(toas)
    if red is None:
        F, ff = fourier_basis(toas, components)
        phi = powerlaw(ff, log10_A, gamma)
        red = F @ (np.sqrt(phi) * rng.standard_normal(2 * components))
    z = (rng.random(n) < theta).astype(np.int64)
    xi = rng.standard_normal(n) if dof is None else rng.standard_t(dof, n)
    r = red + ((1 - z) * toaerrs + z * sigma_out) * xi
    r = r - U @ (U.T @ r)
    return r, z


def at_epochs(raw: dict, seed: int = 1713, theta: float = 0.05, sigma_out: float = 1e-6,
              red_source: str = "powerlaw", name: str = "PSR") -> PulsarData:
    """A pulsar at the epochs / error bars / timing model of ``raw`` (``load_j1713_raw`` or
    ``partim.load_raw`` layout) with synthetic residuals (simulate_data.py:10-39 recipe).

    ``red_source='red.txt'`` adds ``raw['red']`` (the reference's precomputed red-noise
    realisation, interpreted in days as libstempo perturbs ``stoas``) instead
    of a fresh power-law draw.
    """
    mjd = raw["mjd_int"].astype(np.float64) + raw["mjd_frac"]
    toas = mjd * DAY_SEC
    toaerrs = raw["toaerr_us"] * 1e-6
    M = design_matrix(mjd, raw["par"], raw["fit"])
    U = np.linalg.svd(M, full_matrices=False)[0]
    rng = np.random.default_rng(seed)
    red = None
    if red_source == "red.txt":
        if raw.get("red") is None or len(raw["red"]) != len(mjd):
            raise ValueError("red_source='red.txt' needs one red-noise value per TOA")
        red = raw["red"] * DAY_SEC
    r, z = simulate_residuals(toas, toaerrs, U, theta=theta, sigma_out=sigma_out,
                              rng=rng, red=red)
    return PulsarData(name=name, toas=toas, residuals=r, toaerrs=toaerrs, Mmat=M,
                      freqs=raw["freq_mhz"], meta={"z_true": z, "seed": seed,
                                                   "theta": theta})


def j1713(seed: int = 1713, theta: float = 0.05, sigma_out: float = 1e-6,
          red_source: str = "powerlaw") -> PulsarData:
    """J1713+0747 at its 130 real epochs with synthetic residuals (configs 1-2)."""
    return at_epochs(load_j1713_raw(), seed, theta, sigma_out, red_source, "J1713+0747")


def load_partim(par: str, tim: str, red: str | None = None, **kw) -> PulsarData:
    """Any pulsar's tempo2 par/tim pair (gibbs_student_t_amd.partim) at its own epochs,
    error bars and fitted timing model, with synthetic residuals as in ``at_epochs``
    (tempo2 residuals are unavailable offline: parity unpinned)."""
    from . import partim
    raw = partim.load_raw(par, tim, red)
    return at_epochs(raw, name=raw["name"] or "PSR", **kw)


def simulate_data(seed: int, theta: float = 0.05, sigma_out: float = 1e-6,
                  red_source: str = "powerlaw", dof=None):
    """Restatement of simulate_data.py:10-39 on the J1713+0747 epochs.

    Error bars are log-normal ``10^(-7 + 0.2 xi)`` s (simulate_data.py:15).  Returns the
    ``(outlier, no_outlier)`` pair as simulate_data.py writes them: the second drops the
    outlier TOAs (simulate_data.py:35-37), so the two datasets have different n.
    """
    raw = load_j1713_raw()
    mjd = raw["mjd_int"].astype(np.float64) + raw["mjd_frac"]
    toas = mjd * DAY_SEC
    rng = np.random.default_rng(seed)
    err = 10 ** (-7 + rng.standard_normal(len(toas)) * 0.2)
    M = design_matrix(mjd, raw["par"], raw["fit"])
    U = np.linalg.svd(M, full_matrices=False)[0]
    red = raw["red"] * DAY_SEC if red_source == "red.txt" else None
    r, z = simulate_residuals(toas, err, U, theta=theta, sigma_out=sigma_out, rng=rng,
                              red=red, dof=dof)
    out = PulsarData(name="J1713+0747", toas=toas, residuals=r, toaerrs=err, Mmat=M,
                     meta={"z_true": z, "seed": seed, "theta": theta})
    keep = z == 0
    M2 = M[keep]
    U2 = np.linalg.svd(M2, full_matrices=False)[0]
    r2 = r[keep] - U2 @ (U2.T @ r[keep])
    clean = PulsarData(name="J1713+0747", toas=toas[keep], residuals=r2, toaerrs=err[keep],
                       Mmat=M2, meta={"seed": seed, "theta": theta})
    return out, clean


def scaled_synthetic(n: int = 100_000, components: int = 60, ntm: int = 300, seed: int = 5,
                     years: float = 10.0, theta: float = 0.05, sigma_out: float = 1e-6,
                     log10_A: float = -14.0, gamma: float = 4.33) -> PulsarData:
    """BASELINE config 5 ("scaled synthetic: 100k TOAs, 60 red-noise Fourier modes + 300
    timing/DMX columns, m ~ 420") -- not in the reference; built with its recipe:

    TOAs uniform over ``years``, log-normal error bars 10^(-7 + 0.2 xi) s
    (simulate_data.py:15), power-law red noise, Bernoulli(theta) outliers with sigma_out
    (simulate_data.py:24-26), and a random ``ntm``-column timing/DMX design matrix whose
    span is projected out of the residuals (its SVD basis is orthonormal, run_sims.py:22-25).
    """
    rng = np.random.default_rng(seed)
    t0 = 53000.0 * DAY_SEC
    toas = np.sort(t0 + rng.uniform(0.0, years * 365.25 * DAY_SEC, n))
    err = 10 ** (-7 + rng.standard_normal(n) * 0.2)
    tt = (toas - toas.mean()) / (toas.max() - toas.min())
    # a few smooth spin/astrometry-like columns, then random DMX-like columns
    M = [np.ones(n), tt, tt ** 2]
    M += [rng.standard_normal(n) for _ in range(max(0, ntm - 3))]
    M = np.column_stack(M[:ntm])
    U = np.linalg.svd(M, full_matrices=False)[0]
    r, z = simulate_residuals(toas, err, U, theta=theta, sigma_out=sigma_out,
                              log10_A=log10_A, gamma=gamma, components=components, rng=rng)
    return PulsarData(name="SIM", toas=toas, residuals=r, toaerrs=err, Mmat=M,
                      meta={"z_true": z, "seed": seed, "theta": theta})


def multiband(nepochs: int = 60, nsub: int = 3, backends=("ASP", "GUPPI"), seed: int = 1643,
              theta: float = 0.05, sigma_out: float = 1e-6, efac=(1.1, 0.9),
              log10_equad=(-6.6, -7.0), log10_ecorr=(-6.5, -6.8), log10_A: float = -14.0,
              gamma: float = 4.33, components: int = 10, nerr: int = 0) -> PulsarData:
    """A NANOGrav-style multi-backend, multi-band dataset for the general white-noise model
    of the notebook's J1643-1224 run (gibbs_likelihood.ipynb cell 2: efac, equad, ECORR per
    backend, power-law red noise, timing model) -- not in the reference's data, built with
    the simulate_data.py recipe on the first ``nepochs`` J1713+0747 epochs:

    each epoch has ``nsub`` sub-band TOAs at the same arrival time (0.1 s apart, one ECORR
    epoch), the first half of the epochs on ``backends[0]``, the rest on ``backends[1]``;
    white noise ``efac_b sigma`` + ``10^equad_b`` per TOA, ECORR jitter ``10^ecorr_b`` shared
    by an epoch's TOAs, power-law red noise, Bernoulli(theta) outliers, and the timing model
    projected out.  The per-backend true values are in ``meta``.  ``nerr`` > 0: every TOA's
    error bar is one of ``nerr`` values (a few noise classes per backend, as a receiver's
    quantised template-fit errors give) instead of log-normal."""
    raw = load_j1713_raw()
    mjd0 = (raw["mjd_int"].astype(np.float64) + raw["mjd_frac"])[:nepochs]
    rng = np.random.default_rng(seed)
    mjd = np.repeat(mjd0, nsub) + np.tile(np.arange(nsub) * 0.1 / DAY_SEC, nepochs)
    toas = mjd * DAY_SEC
    n = len(toas)
    ep = np.repeat(np.arange(nepochs), nsub)
    bk = (ep >= nepochs // 2).astype(np.int64)
    labels = np.array(backends)[bk]
    err = 10 ** (-7 + rng.standard_normal(n) * 0.2)
    if nerr > 0:
        err = 10 ** (-7 + 0.2 * (rng.integers(0, nerr, size=n) - (nerr - 1) / 2.0))
    M = design_matrix(mjd, raw["par"], raw["fit"])
    U = np.linalg.svd(M, full_matrices=False)[0]
    F, ff = fourier_basis(toas, components)
    red = F @ (np.sqrt(powerlaw(ff, log10_A, gamma)) * rng.standard_normal(2 * components))
    ef, eq, ec = (np.asarray(v, dtype=np.float64)[bk] for v in (efac, log10_equad, log10_ecorr))
    jitter = (10 ** np.asarray(log10_ecorr)[(np.arange(nepochs) >= nepochs // 2).astype(int)]
              * rng.standard_normal(nepochs))[ep]
    white = np.sqrt((ef * err) ** 2 + 10 ** (2 * eq)) * rng.standard_normal(n)
    z = (rng.random(n) < theta).astype(np.int64)
    r = red + jitter + np.where(z == 1, sigma_out * rng.standard_normal(n), white)
    r = r - U @ (U.T @ r)
    return PulsarData(name="MB", toas=toas, residuals=r, toaerrs=err, Mmat=M, backends=labels,
                      meta={"z_true": z, "seed": seed, "theta": theta, "efac": efac,
                            "log10_equad": log10_equad, "log10_ecorr": log10_ecorr,
                            "epoch": ep})


__all__ = ["load_j1713_raw", "multiband", "scaled_synthetic", "design_matrix", "simulate_residuals", "j1713",
           "at_epochs", "load_partim", "simulate_data", "FYR"]
