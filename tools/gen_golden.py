"""Generate golden vectors by running the REFERENCE sampler (/root/reference/gibbs.py).

Runs only in the build container (the reference never travels).  Outputs small .npz
fixtures under tests/golden/ that pin both the CPU oracle and the HIP path:

* the reference's chain arrays (chain, bchain, zchain, poutchain, thetachain, alphachain,
  dfchain) for a short run per run_sims.py model (run_sims.py:89-107), seeded;
* the variate tape each sweep consumed (MH uniforms / index / jump / accept uniforms,
  b normals, beta value, binomial uniforms, gamma values, dof-choice uniform), recovered
  from the legacy MT19937 state around each call;
* every likelihood evaluation (x, value) of the white and hyper MH blocks;
* for each b draw: the reference's SVD mean, its draw term Li @ xi, the Cholesky mean
  ``cho_solve(cho_factor(Sigma), d)`` (gibbs.py:321-322) and cond(Sigma).

The only shim is Python-2 ``map`` -> list, set on the imported
module; nothing of the reference is copied.
"""
from __future__ import annotations

import builtins
import os
import sys
import warnings

import numpy as np
import scipy.linalg as sl
import scipy.stats

sys.dont_write_bytecode = True
sys.path.insert(0, "/root/reference")
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)

import gibbs as refgibbs  # noqa: E402  (the reference)

from gibbs_student_t_amd import data as gdata  # noqa: E402
from gibbs_student_t_amd.model import PTA  # noqa: E402

refgibbs.map = lambda f, *a: list(builtins.map(f, *a))
warnings.filterwarnings("ignore", category=DeprecationWarning)

OUTDIR = os.path.join(ROOT, "tests", "golden")
RS = np.random.mtrand._rand

MODELS = {
    # run_sims.py:89-107
    "vvh17": dict(model="vvh17", vary_df=False, theta_prior="uniform", vary_alpha=False,
                  alpha=1e10, pspin=0.00457),
    "uniform": dict(model="mixture", vary_df=True, theta_prior="uniform"),
    "beta": dict(model="mixture", vary_df=True, theta_prior="beta"),
    "gaussian": dict(model="gaussian", vary_df=True, theta_prior="beta"),
    "t": dict(model="t", vary_df=True, theta_prior="beta"),
}


def _same_state(a, b):
    return (a[0] == b[0] and np.array_equal(a[1], b[1]) and a[2] == b[2]
            and a[3] == b[3] and a[4] == b[4])


class Rec:
    stage = None
    sweeps = []

    @classmethod
    def cur(cls):
        return cls.sweeps[-1]


_orig = {
    "choice": np.random.choice, "randn": np.random.randn, "rand": np.random.rand,
    "beta": scipy.stats.beta.rvs, "binom": scipy.stats.binom.rvs,
    "gamma": scipy.stats.gamma.rvs,
}


def _uniform_of(call, *a, **k):
    """Run ``call`` and recover the single uniform it consumed from the MT state."""
    st0 = RS.get_state()
    val = call(*a, **k)
    st1 = RS.get_state()
    RS.set_state(st0)
    u = RS.random_sample()
    assert _same_state(RS.get_state(), st1), "call consumed more than one uniform"
    return val, u


def rec_choice(a, size=None, replace=True, p=None):
    ev = Rec.cur()
    if p is not None:
        val, u = _uniform_of(_orig["choice"], a, size=size, replace=replace, p=p)
        if Rec.stage == "df":
            ev["df_u"] = u
        else:
            ev[f"{Rec.stage}_u"].append(u)
        return val
    val = _orig["choice"](a, size=size, replace=replace, p=p)
    ev[f"{Rec.stage}_idx"].append(int(np.asarray(val).ravel()[0]))
    return val


def rec_randn(*shape):
    val = _orig["randn"](*shape)
    ev = Rec.cur()
    if Rec.stage in ("white", "hyper"):
        ev[f"{Rec.stage}_xi"].append(float(val[0]))
    elif Rec.stage == "b":
        ev["b_xi"] = np.array(val)
    return val


def rec_rand(*shape):
    val = _orig["rand"](*shape)
    Rec.cur()[f"{Rec.stage}_acc"].append(float(val))
    return val


def rec_beta(*a, **k):
    val = _orig["beta"](*a, **k)
    Rec.cur()["beta"] = float(val)
    return val


def rec_binom(nn, p, *a, **k):
    st0 = RS.get_state()
    z = _orig["binom"](nn, p, *a, **k)
    st1 = RS.get_state()
    RS.set_state(st0)
    p = np.asarray(p, dtype=np.float64)
    u = np.full(len(p), np.nan)
    for i, pi in enumerate(p):
        if pi != 0.0:
            u[i] = RS.random_sample()
    assert _same_state(RS.get_state(), st1), "binomial uniform recovery failed"
    RS.set_state(st1)
    Rec.cur()["z_u"] = u
    return z


def rec_gamma(*a, **k):
    val = _orig["gamma"](*a, **k)
    Rec.cur()["gamma"] = np.array(val, dtype=np.float64)
    return val


class RecordingGibbs(refgibbs.Gibbs):
    def update_white_params(self, xs):
        Rec.sweeps.append({k: [] for k in ("white_u", "white_idx", "white_xi", "white_acc",
                                          "hyper_u", "hyper_idx", "hyper_xi", "hyper_acc",
                                          "white_lnl_x", "white_lnl", "hyper_lnl_x",
                                          "hyper_lnl")})
        Rec.stage = "white"
        out = super().update_white_params(xs)
        Rec.cur()["x_white"] = np.array(out)
        return out

    def update_hyper_params(self, xs):
        Rec.stage = "hyper"
        return super().update_hyper_params(xs)

    def update_b(self, xs):
        Rec.stage = "b"
        b = super().update_b(xs)
        params = self.map_params(xs)
        phiinv = self.pta.get_phiinv(params, logdet=False)[0]
        Sigma = self.TNT + np.diag(phiinv)
        u, s, _ = sl.svd(Sigma)
        mn = np.dot(u, np.dot(u.T, self.d) / s)
        Li = u * np.sqrt(1 / s)
        ev = Rec.cur()
        ev["b_delta"] = np.dot(Li, ev["b_xi"])
        ev["b_mean_svd"] = mn
        ev["b_mean_chol"] = sl.cho_solve(sl.cho_factor(Sigma), self.d)
        ev["b_cond"] = float(np.linalg.cond(Sigma))
        ev["b_ref"] = np.array(b)
        assert np.array_equal(b, mn + np.dot(Li, ev["b_xi"]))
        return b

    def update_theta(self, xs):
        Rec.stage = "theta"
        return super().update_theta(xs)

    def update_z(self, xs):
        Rec.stage = "z"
        return super().update_z(xs)

    def update_alpha(self, xs):
        Rec.stage = "alpha"
        return super().update_alpha(xs)

    def update_df(self, xs):
        Rec.stage = "df"
        return super().update_df(xs)

    def get_lnlikelihood_white(self, xs):
        v = super().get_lnlikelihood_white(xs)
        ev = Rec.cur()
        ev["white_lnl_x"].append(np.array(xs, dtype=np.float64))
        ev["white_lnl"].append(float(v))
        return v

    def get_lnlikelihood(self, xs):
        v = super().get_lnlikelihood(xs)
        ev = Rec.cur()
        ev["hyper_lnl_x"].append(np.array(xs, dtype=np.float64))
        ev["hyper_lnl"].append(float(v))
        return v


def _install():
    np.random.choice = rec_choice
    np.random.randn = rec_randn
    np.random.rand = rec_rand
    scipy.stats.beta.rvs = rec_beta
    scipy.stats.binom.rvs = rec_binom
    scipy.stats.gamma.rvs = rec_gamma


def _uninstall():
    np.random.choice = _orig["choice"]
    np.random.randn = _orig["randn"]
    np.random.rand = _orig["rand"]
    for nm in ("beta", "binom", "gamma"):
        if nm in getattr(scipy.stats, nm).__dict__:
            del getattr(scipy.stats, nm).__dict__["rvs"]


def pack_tape(sweeps, n, m, P):
    S = len(sweeps)
    T = {
        "white_u": np.full((S, 20), np.nan), "white_idx": np.full((S, 20), -1, np.int64),
        "white_xi": np.full((S, 20), np.nan), "white_acc": np.full((S, 20), np.nan),
        "hyper_u": np.full((S, 10), np.nan), "hyper_idx": np.full((S, 10), -1, np.int64),
        "hyper_xi": np.full((S, 10), np.nan), "hyper_acc": np.full((S, 10), np.nan),
        "b_xi": np.full((S, m), np.nan), "b_delta": np.full((S, m), np.nan),
        "b_mean_svd": np.full((S, m), np.nan), "b_mean_chol": np.full((S, m), np.nan),
        "b_ref": np.full((S, m), np.nan), "b_cond": np.full(S, np.nan),
        "beta": np.full(S, np.nan), "z_u": np.full((S, n), np.nan),
        "gamma": np.full((S, n), np.nan), "df_u": np.full(S, np.nan),
        "x_white": np.full((S, P), np.nan),
        "white_lnl_x": np.full((S, 21, P), np.nan), "white_lnl": np.full((S, 21), np.nan),
        "hyper_lnl_x": np.full((S, 11, P), np.nan), "hyper_lnl": np.full((S, 11), np.nan),
    }
    for i, ev in enumerate(sweeps):
        for stage, k in (("white", 20), ("hyper", 10)):
            T[f"{stage}_u"][i] = ev[f"{stage}_u"]
            T[f"{stage}_xi"][i] = ev[f"{stage}_xi"]
            T[f"{stage}_acc"][i] = ev[f"{stage}_acc"]
            T[f"{stage}_idx"][i] = ev[f"{stage}_idx"]
            T[f"{stage}_lnl_x"][i] = np.array(ev[f"{stage}_lnl_x"])
            T[f"{stage}_lnl"][i] = ev[f"{stage}_lnl"]
        T["x_white"][i] = ev["x_white"]
        for key in ("b_xi", "b_delta", "b_mean_svd", "b_mean_chol", "b_ref", "b_cond",
                    "beta", "z_u", "gamma", "df_u"):
            if key in ev:
                T[key][i] = ev[key]
    return T


def run_one(pta, name, kw, seed, niter, x0=None):
    Rec.sweeps = []
    np.random.seed(seed)
    xs = pta.sample_params() if x0 is None else np.array(x0, dtype=np.float64)
    g = RecordingGibbs(pta, **kw)
    _install()
    try:
        g.sample(xs, niter=niter)
    finally:
        _uninstall()
    n, m, P = pta.n, pta.m, len(xs)
    tape = pack_tape(Rec.sweeps, n, m, P)
    out = dict(xs=xs, seed=seed, niter=niter, chain=g.chain, bchain=g.bchain,
               zchain=g.zchain, poutchain=g.poutchain, thetachain=g.thetachain,
               alphachain=g.alphachain, dfchain=g.dfchain,
               final_b=g._b, final_z=np.asarray(g._z, dtype=np.float64),
               final_alpha=g._alpha, final_pout=g._pout, final_theta=g._theta,
               final_df=float(g.tdf), prior_draw=int(x0 is None))
    out.update({f"tape_{k}": v for k, v in tape.items()})
    return out


def dataset_arrays(pta, psr):
    out = dict(toas=psr.toas, residuals=psr.residuals, toaerrs=psr.toaerrs, Mmat=psr.Mmat,
               T=pta.T, Ffreqs=pta.Ffreqs, components=pta.components,
               tm_weight=pta.tm_weight, names=np.array(pta.param_names))
    if pta.nbackend > 1 or pta.n_ecorr or getattr(pta, "has_ecorr", False):
        # general white-noise model (per-backend parameters, ECORR basis columns)
        out.update(backends=np.asarray(psr.backends).astype(str), selection=pta.selection,
                   n_ecorr=pta.n_ecorr, ecorr_backend=pta.ecorr_backend,
                   efac_varied=int(pta.efac_const is None),
                   log10_ecorr=np.array([-8.5, -5.0] if pta.n_ecorr else []))
    return out


def simclean(niter=12):
    """simulate_data.py's no_outlier twin (outlier TOAs deleted, simulate_data.py:35-37):
    n < 130, so a batch with the outlier dataset is ragged."""
    sim, clean = gdata.simulate_data(seed=7, theta=0.1)
    pta5 = PTA(clean)
    np.savez_compressed(os.path.join(OUTDIR, "simclean_dataset.npz"),
                        **dataset_arrays(pta5, clean))
    for name in ("beta", "vvh17"):
        out = run_one(pta5, name, MODELS[name], seed=778, niter=niter, x0=[4.33, -14.0, -7.6])
        out["model_kw"] = np.array(repr(MODELS[name]))
        np.savez_compressed(os.path.join(OUTDIR, f"ref_simclean_{name}_fixed.npz"), **out)
        print("simclean", name, "n", pta5.n, "cond:", np.nanmax(out["tape_b_cond"]),
              file=sys.stderr)


def scaled(niter=6):
    """A mid-size cut of BASELINE config 5 (gdata.scaled_synthetic): n = 1500 TOAs,
    40 red-noise components (80 Fourier columns) + 100 timing/DMX columns, m = 180 --
    beyond the register-resident kernel, exercising the multi-kernel large path."""
    psr = gdata.scaled_synthetic(n=1500, components=40, ntm=100, seed=11)
    pta6 = PTA(psr, components=40)
    np.savez_compressed(os.path.join(OUTDIR, "scaled_dataset.npz"), **dataset_arrays(pta6, psr))
    for name in ("beta", "t"):
        out = run_one(pta6, name, MODELS[name], seed=3300 + len(name), niter=niter,
                      x0=[4.33, -14.0, -7.6])
        out["model_kw"] = np.array(repr(MODELS[name]))
        np.savez_compressed(os.path.join(OUTDIR, f"ref_scaled_{name}_fixed.npz"), **out)
        print("scaled", name, "n", pta6.n, "m", pta6.m, "cond:",
              np.nanmax(out["tape_b_cond"]), file=sys.stderr)


def configs34(niter=12):
    """Datasets of BASELINE configs 3 and 4 run through the reference.

    * ``c3``: the config-3 pulsar -- simulate_data.py restatement with 5% outliers and the
      reference's red.txt red-noise realisation (bench.py --config 3 uses seed 2017).
    * ``c4t``: a config-4 Student-t white-noise dataset -- the run_sims grid's first
      (theta = 0.05, dof = 4) realisation, seeded exactly as run_sims.build_grid seeds it.
    """
    c3, _ = gdata.simulate_data(seed=2017, theta=0.05, red_source="red.txt")
    sd = int(np.random.SeedSequence([2017, 0, 0, 1]).generate_state(1)[0])
    c4, _ = gdata.simulate_data(sd, theta=0.05, dof=4.0)
    for tag, psr, models in (("c3", c3, ("beta", "t", "uniform")),
                             ("c4t", c4, ("beta", "t", "gaussian"))):
        pta_c = PTA(psr)
        np.savez_compressed(os.path.join(OUTDIR, f"{tag}_dataset.npz"),
                            **dataset_arrays(pta_c, psr))
        for j, name in enumerate(models):
            out = run_one(pta_c, name, MODELS[name], seed=5100 + 31 * j + len(tag),
                          niter=niter, x0=[4.33, -14.0, -7.6])
            out["model_kw"] = np.array(repr(MODELS[name]))
            np.savez_compressed(os.path.join(OUTDIR, f"ref_{tag}_{name}_fixed.npz"), **out)
            print(tag, name, "n", pta_c.n, "cond:", np.nanmax(out["tape_b_cond"]),
                  file=sys.stderr)


def shapes(niter=12):
    """Other model shapes on the J1713+0747 epochs (register-resident instances padded with
    unit-prior dummy columns):

    * ``c20``: 20 red-noise components (the notebook's count, gibbs_likelihood.ipynb cell 2)
      with the 14 timing-model columns;
    * ``tm22``: 20 components with 22 timing-model columns (the 14 plus 8 DMX-like
      piecewise-constant offsets over the 5 years), i.e. 17..24 columns -> 3 TM panels.
    """
    import copy
    psr = gdata.j1713(seed=1713, theta=0.05)
    pta_a = PTA(psr, components=20)
    np.savez_compressed(os.path.join(OUTDIR, "c20_dataset.npz"), **dataset_arrays(pta_a, psr))
    psr22 = copy.deepcopy(psr)
    t = psr.toas
    edges = np.linspace(t.min(), t.max() + 1.0, 9)
    dmx = np.stack([((t >= a) & (t < b)).astype(float) for a, b in zip(edges[:-1], edges[1:])],
                   axis=1)
    psr22.Mmat = np.column_stack([psr.Mmat, dmx])
    pta_b = PTA(psr22, components=20)
    assert pta_b.ntm == 22, pta_b.ntm
    np.savez_compressed(os.path.join(OUTDIR, "tm22_dataset.npz"), **dataset_arrays(pta_b, psr22))
    for tag, pta_s, models in (("c20", pta_a, ("beta", "t", "vvh17")),
                               ("tm22", pta_b, ("beta", "uniform"))):
        for j, name in enumerate(models):
            out = run_one(pta_s, name, MODELS[name], seed=6100 + 17 * j + len(tag),
                          niter=niter, x0=[4.33, -14.0, -7.6])
            out["model_kw"] = np.array(repr(MODELS[name]))
            np.savez_compressed(os.path.join(OUTDIR, f"ref_{tag}_{name}_fixed.npz"), **out)
            print(tag, name, "m", pta_s.m, "cond:", np.nanmax(out["tape_b_cond"]),
                  file=sys.stderr)


def general(niter=12):
    """The general white-noise model of the notebook's J1643-1224 run (gibbs_likelihood.ipynb
    cell 2: efac, equad, ECORR basis, power-law red noise, timing model) on a multi-band,
    two-backend dataset (gdata.multiband: 60 J1713 epochs x 3 sub-band TOAs, ASP then GUPPI):

    * ``mb``: ``selection="backend"``, varied efac, equad and ECORR per backend: P = 8
      (white index set of 4, hyper set of 4: the two ecorr, log10_A, gamma, gibbs.py:64-77),
      10 red-noise components, 60 ECORR epoch columns (m = 94);
    * ``mbn``: ``no_selection`` as the notebook runs it: P = 5 (efac, ecorr, equad, gamma,
      log10_A), one ECORR prior for all 60 epochs.
    """
    psr = gdata.multiband()
    pta_b = PTA(psr, components=10, efac=(0.2, 10.0), selection="backend",
                log10_ecorr=(-8.5, -5.0))
    pta_n = PTA(psr, components=10, efac=(0.2, 10.0), log10_ecorr=(-8.5, -5.0))
    x0b = [1.1, -6.5, -6.6, 0.9, -6.8, -7.0, 4.33, -14.0]
    x0n = [1.0, 4.33, -14.0, -6.6, -6.8]    # efac, gamma, log10_A, log10_ecorr, log10_equad
    for tag, pta_g, x0, models in (("mb", pta_b, x0b, ("beta", "t", "gaussian")),
                                   ("mbn", pta_n, x0n, ("beta", "vvh17"))):
        np.savez_compressed(os.path.join(OUTDIR, f"{tag}_dataset.npz"),
                            **dataset_arrays(pta_g, psr))
        for j, name in enumerate(models):
            out = run_one(pta_g, name, MODELS[name], seed=7300 + 13 * j + len(tag),
                          niter=niter, x0=x0)
            out["model_kw"] = np.array(repr(MODELS[name]))
            np.savez_compressed(os.path.join(OUTDIR, f"ref_{tag}_{name}_fixed.npz"), **out)
            print(tag, name, "P", len(x0), "m", pta_g.m, "cond:",
                  np.nanmax(out["tape_b_cond"]), file=sys.stderr)


def small_ecorr(niter=12):
    """The general white-noise model with a hyper block the register-resident large-path
    kernel takes (lg_hyper_reg: nf + n_ecorr <= 62): gdata.multiband with 24 epochs x 3
    sub-band TOAs (n = 72), 10 red-noise components and 24 ECORR epochs (20 + 24 = 44 hyper
    columns, m = 58); ``ecb``: per-backend efac / equad / ECORR (P = 8), ``ecn``: one of each
    (P = 5), as ``general`` (lg_hyper_reg's ECORR branches)."""
    psr = gdata.multiband(nepochs=24, nsub=3, seed=2443)
    pta_b = PTA(psr, components=10, efac=(0.2, 10.0), selection="backend",
                log10_ecorr=(-8.5, -5.0))
    pta_n = PTA(psr, components=10, efac=(0.2, 10.0), log10_ecorr=(-8.5, -5.0))
    x0b = [1.1, -6.5, -6.6, 0.9, -6.8, -7.0, 4.33, -14.0]
    x0n = [1.0, 4.33, -14.0, -6.6, -6.8]
    for tag, pta_g, x0, models in (("ecb", pta_b, x0b, ("beta", "uniform")),
                                   ("ecn", pta_n, x0n, ("t", "vvh17"))):
        np.savez_compressed(os.path.join(OUTDIR, f"{tag}_dataset.npz"),
                            **dataset_arrays(pta_g, psr))
        for j, name in enumerate(models):
            out = run_one(pta_g, name, MODELS[name], seed=7700 + 13 * j + len(tag),
                          niter=niter, x0=x0)
            out["model_kw"] = np.array(repr(MODELS[name]))
            np.savez_compressed(os.path.join(OUTDIR, f"ref_{tag}_{name}_fixed.npz"), **out)
            print(tag, name, "P", len(x0), "m", pta_g.m, "cond:",
                  np.nanmax(out["tape_b_cond"]), file=sys.stderr)


def ecorr_classes(niter=12):
    """``ecq``: the ``ecb`` model (per-backend efac / equad / ECORR, 20 Fourier + 24 ECORR
    columns) on a pulsar whose error bars take two values (gdata.multiband nerr = 2): four
    noise classes (error bar x backend), so the persistent kernel's general white-noise
    instances take their noise-class likelihood and low-rank Gram paths (gst_kernel.hpp
    lnl_white / gram_and_tm with GEN)."""
    psr = gdata.multiband(nepochs=24, nsub=3, seed=2445, nerr=2)
    pta_q = PTA(psr, components=10, efac=(0.2, 10.0), selection="backend",
                log10_ecorr=(-8.5, -5.0))
    x0 = [1.1, -6.5, -6.6, 0.9, -6.8, -7.0, 4.33, -14.0]
    np.savez_compressed(os.path.join(OUTDIR, "ecq_dataset.npz"), **dataset_arrays(pta_q, psr))
    for j, name in enumerate(("beta", "t")):
        out = run_one(pta_q, name, MODELS[name], seed=7900 + 13 * j, niter=niter, x0=x0)
        out["model_kw"] = np.array(repr(MODELS[name]))
        np.savez_compressed(os.path.join(OUTDIR, f"ref_ecq_{name}_fixed.npz"), **out)
        print("ecq", name, "P", len(x0), "m", pta_q.m, "cond:",
              np.nanmax(out["tape_b_cond"]), file=sys.stderr)


def ecorr_big(niter=12):
    """``ebig``: per-backend efac / equad / ECORR on 130 epochs x 2 sub-band TOAs (n = 260):
    20 Fourier + 130 ECORR columns (m = 164), a red-noise / ECORR block past the large path's
    LDS-resident one (gst_large.hpp HYPER_LDS_MAX = 138), which lg_hyper<true> factors in
    global memory -- NANOGrav-style pulsars carry hundreds of ECORR epochs."""
    psr = gdata.multiband(nepochs=130, nsub=2, seed=2446)
    pta_e = PTA(psr, components=10, efac=(0.2, 10.0), selection="backend",
                log10_ecorr=(-8.5, -5.0))
    x0 = [1.1, -6.5, -6.6, 0.9, -6.8, -7.0, 4.33, -14.0]
    np.savez_compressed(os.path.join(OUTDIR, "ebig_dataset.npz"), **dataset_arrays(pta_e, psr))
    for j, name in enumerate(("beta", "t")):
        out = run_one(pta_e, name, MODELS[name], seed=8300 + 13 * j, niter=niter, x0=x0)
        out["model_kw"] = np.array(repr(MODELS[name]))
        np.savez_compressed(os.path.join(OUTDIR, f"ref_ebig_{name}_fixed.npz"), **out)
        print("ebig", name, "P", len(x0), "m", pta_e.m, "n_ecorr", pta_e.n_ecorr, "cond:",
              np.nanmax(out["tape_b_cond"]), file=sys.stderr)


def j1713_backends(niter=12):
    """``jb``: the headline pulsar (J1713+0747's 130 epochs, run_sims' 30 red-noise
    components and 14-column timing model, m = 74) with per-backend efac / equad and no
    ECORR: the first half of the epochs on ASP, the rest on GUPPI (P = 6).  J1713's error
    bars are all one value, so the model has two noise classes (backend x error bar) and
    the persistent kernel's general white-noise instances take their class paths."""
    psr = gdata.j1713(seed=1714, theta=0.05)
    order = np.argsort(psr.toas)
    labels = np.empty(psr.n, dtype="<U5")
    labels[order] = np.where(np.arange(psr.n) < psr.n // 2, "ASP", "GUPPI")
    psr.backends = labels
    pta = PTA(psr, efac=(0.2, 10.0), selection="backend")
    x0 = [1.1, -6.5, 0.9, -7.0, 4.33, -14.0]   # ASP efac, equad, GUPPI efac, equad, gamma, A
    np.savez_compressed(os.path.join(OUTDIR, "jb_dataset.npz"), **dataset_arrays(pta, psr))
    for j, name in enumerate(("beta", "uniform")):
        out = run_one(pta, name, MODELS[name], seed=8500 + 13 * j, niter=niter, x0=x0)
        out["model_kw"] = np.array(repr(MODELS[name]))
        np.savez_compressed(os.path.join(OUTDIR, f"ref_jb_{name}_fixed.npz"), **out)
        print("jb", name, "P", len(x0), "m", pta.m, "cond:",
              np.nanmax(out["tape_b_cond"]), file=sys.stderr)


def mid(niter=12):
    """A mid-size pulsar for the register-resident kernel's wide TOA instances (NS = 6, 8
    slots of 64 TOAs): 130 J1713+0747 epochs x 3 sub-band TOAs (gdata.multiband, one
    backend's labels ignored), n = 390, the classic run_sims model (30 components)."""
    psr = gdata.multiband(nepochs=130, nsub=3, seed=390)
    pta_m = PTA(psr)
    np.savez_compressed(os.path.join(OUTDIR, "mid_dataset.npz"), **dataset_arrays(pta_m, psr))
    for j, name in enumerate(("beta", "t")):
        out = run_one(pta_m, name, MODELS[name], seed=8100 + 11 * j, niter=niter,
                      x0=[4.33, -14.0, -7.6])
        out["model_kw"] = np.array(repr(MODELS[name]))
        np.savez_compressed(os.path.join(OUTDIR, f"ref_mid_{name}_fixed.npz"), **out)
        print("mid", name, "n", pta_m.n, "cond:", np.nanmax(out["tape_b_cond"]), file=sys.stderr)


def wide(niter=12):
    """A wider mid-size pulsar for the register-resident kernel's 16-slot instance (n <= 1024):
    130 J1713+0747 epochs x 7 sub-band TOAs (gdata.multiband, one backend's labels ignored),
    n = 910, the classic run_sims model (30 components)."""
    psr = gdata.multiband(nepochs=130, nsub=7, seed=910)
    pta_w = PTA(psr)
    np.savez_compressed(os.path.join(OUTDIR, "wide_dataset.npz"), **dataset_arrays(pta_w, psr))
    for j, name in enumerate(("beta", "t")):
        out = run_one(pta_w, name, MODELS[name], seed=9100 + 11 * j, niter=niter,
                      x0=[4.33, -14.0, -7.6])
        out["model_kw"] = np.array(repr(MODELS[name]))
        np.savez_compressed(os.path.join(OUTDIR, f"ref_wide_{name}_fixed.npz"), **out)
        print("wide", name, "n", pta_w.n, "cond:", np.nanmax(out["tape_b_cond"]),
              file=sys.stderr)


def main():
    os.makedirs(OUTDIR, exist_ok=True)
    if "--only-wide" in sys.argv:
        wide(12)
        return
    if "--only-general" in sys.argv:
        general(12)
        return
    if "--only-small-ecorr" in sys.argv:
        small_ecorr(12)
        return
    if "--only-ecorr-classes" in sys.argv:
        ecorr_classes(12)
        return
    if "--only-ecorr-big" in sys.argv:
        ecorr_big(12)
        return
    if "--only-j1713-backends" in sys.argv:
        j1713_backends(12)
        return
    if "--only-mid" in sys.argv:
        mid(12)
        return
    if "--only-shapes" in sys.argv:
        shapes(12)
        return
    niter = 12
    if "--only-simclean" in sys.argv:
        simclean(niter)
        return
    if "--only-scaled" in sys.argv:
        scaled()
        return
    if "--only-configs34" in sys.argv:
        configs34(niter)
        return
    psr = gdata.j1713(seed=1713, theta=0.05)
    pta = PTA(psr)
    np.savez_compressed(os.path.join(OUTDIR, "j1713_dataset.npz"), **dataset_arrays(pta, psr))
    for i, (name, kw) in enumerate(MODELS.items()):
        for tag, x0 in (("prior", None), ("fixed", [4.33, -14.0, -7.6])):
            out = run_one(pta, name, kw, seed=1000 + 17 * i + (tag == "fixed"),
                          niter=niter, x0=x0)
            out["model_kw"] = np.array(repr(kw))
            fn = os.path.join(OUTDIR, f"ref_{name}_{tag}.npz")
            np.savez_compressed(fn, **out)
            print(name, tag, "cond(b):", np.nanmax(out["tape_b_cond"]),
                  "redraws:", int(np.sum(~np.isnan(out["tape_b_cond"]))), file=sys.stderr)
    # varied efac (notebook-style, gibbs_likelihood.ipynb cell 2): two white parameters,
    # so the white index draw is exercised
    pta2 = PTA(psr, efac=(0.2, 10.0))
    np.savez_compressed(os.path.join(OUTDIR, "j1713_dataset_efac.npz"),
                        **dataset_arrays(pta2, psr))
    out = run_one(pta2, "beta", MODELS["beta"], seed=4242, niter=niter,
                  x0=[1.1, 4.33, -14.0, -7.6])
    out["model_kw"] = np.array(repr(MODELS["beta"]))
    np.savez_compressed(os.path.join(OUTDIR, "ref_beta_efac_fixed.npz"), **out)
    print("efac fixed cond:", np.nanmax(out["tape_b_cond"]), file=sys.stderr)
    # simulate_data.py-style pulsar: log-normal error bars (every TOA its own sigma)
    sim, _ = gdata.simulate_data(seed=7, theta=0.1)
    pta3 = PTA(sim)
    np.savez_compressed(os.path.join(OUTDIR, "sim_dataset.npz"), **dataset_arrays(pta3, sim))
    for name in ("beta", "t"):
        out = run_one(pta3, name, MODELS[name], seed=777, niter=niter, x0=[4.33, -14.0, -7.6])
        out["model_kw"] = np.array(repr(MODELS[name]))
        np.savez_compressed(os.path.join(OUTDIR, f"ref_sim_{name}_fixed.npz"), **out)
        print("sim", name, "cond:", np.nanmax(out["tape_b_cond"]), file=sys.stderr)
    # two backends: J1713 epochs with alternating 40 ns / 100 ns error bars (2 noise classes)
    tb = gdata.j1713(seed=1713, theta=0.05)
    tb.toaerrs = np.where(np.arange(tb.n) % 2 == 0, 4e-8, 1e-7)
    pta4 = PTA(tb)
    np.savez_compressed(os.path.join(OUTDIR, "twob_dataset.npz"), **dataset_arrays(pta4, tb))
    out = run_one(pta4, "uniform", MODELS["uniform"], seed=31, niter=niter,
                  x0=[4.33, -14.0, -7.6])
    out["model_kw"] = np.array(repr(MODELS["uniform"]))
    np.savez_compressed(os.path.join(OUTDIR, "ref_twob_uniform_fixed.npz"), **out)
    simclean(niter)
    scaled()
    configs34(niter)
    shapes(niter)
    general(niter)
    small_ecorr(niter)
    ecorr_classes(niter)
    ecorr_big(niter)
    j1713_backends(niter)
    mid(niter)
    wide(niter)


if __name__ == "__main__":
    main()
