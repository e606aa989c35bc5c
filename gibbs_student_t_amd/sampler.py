"""Drop-in ``Gibbs`` sampler (reference: /root/reference/gibbs.py, class Gibbs, :8-385).

Same constructor, same public methods and attributes; every sweep runs on the GPU through
libgst.so.  Extra keyword-only options: ``nchains`` (independent chains batched on the GPU;
chain arrays gain a leading chain axis when > 1), ``seed`` (Philox key), ``device``,
``record_every`` (thin the chain arrays) and ``chunk`` (sweeps per kernel launch).

Differences from the reference, all documented in DESIGN.md:
* ``update_b`` recomputes T^T N^-1 T from the current state; the reference reuses whatever
  TNT/d its last likelihood call cached (gibbs.py:159-161);
* variates come from on-device Philox4x32-10 instead of numpy's MT19937 stream, so chains
  are distributionally -- not bitwise -- equal to the reference's for the same seed;
* the b draw uses the Cholesky square root (mean = cho_solve(Sigma, d), the reference's own
  expression at gibbs.py:321-322) instead of the SVD one at gibbs.py:169-171 -- except where
  Sigma is beyond fp64 resolution (vvh17's all-outlier start): there the reference's SVD
  returns the small eigenvalues at LAPACK's rounding floor and the kernel draws from
  Sigma + f I instead (the SVD noise floor, include/gst.h gst_sweep; ``exact_bdraw=True``
  turns it off).
"""
from __future__ import annotations

import os
import sys
import time

import numpy as np
import scipy.special

from . import _abi
from .native import STATE_KEYS, NativeSampler


class Gibbs:
    def __init__(self, pta, model="gaussian", tdf=4, m=0.01, vary_df=True,
                 theta_prior="beta", vary_alpha=True, alpha=1e10, pspin=None, *,
                 nchains=1, seed=None, device=0, record_every=1, chunk=512, verbose=False,
                 exact_bdraw=False):
        # gibbs.py:13-51.  exact_bdraw: draw b exactly from Sigma also where it is beyond fp64
        # resolution, instead of at the reference's SVD noise floor (include/gst.h gst_sweep)
        self.pta = pta
        self.mp = m
        self.theta_prior = theta_prior
        self.pspin = pspin
        self.vary_df = vary_df
        self.vary_alpha = vary_alpha
        self._residuals = self.pta.get_residuals()[0]
        self._lmodel = model
        self.nchains = int(nchains)
        self.record_every = int(record_every)
        self.chunk = int(chunk)
        self.verbose = verbose
        self.seed = int.from_bytes(os.urandom(8), "little") if seed is None else int(seed)
        self._sweep_counter = 0
        C, n = self.nchains, len(self._residuals)
        mcols = self.pta.get_basis()[0].shape[1]
        self.TNT = None
        self.d = None
        self._b_all = np.zeros((C, mcols))
        self._pout_all = np.zeros((C, n))
        z0 = 1.0 if model in ("t", "mixture", "vvh17") else 0.0
        self._z_all = np.full((C, n), z0)
        self._alpha_all = np.full((C, n), alpha if not vary_alpha else 1.0)
        self._theta_all = np.full(C, float(m))
        self._tdf_all = np.full(C, float(tdf))
        cfg = dict(model=model, tdf=tdf, m=m, vary_df=vary_df, theta_prior=theta_prior,
                   vary_alpha=vary_alpha, alpha=alpha, pspin=pspin)
        self._cfg = dict(cfg, exact_bdraw=bool(exact_bdraw))
        self._x_all = None
        self._counter_at_sample = None      # Philox counter when sample() last returned
        self._native = NativeSampler(pta, cfg, device)
        self._native.set_debug(exact_bdraw=exact_bdraw)
        self._native.alloc(C)

    # ---- reference attribute names (chain 0 view when nchains == 1) -----------------
    def _view(self, a):
        return a[0] if self.nchains == 1 else a

    def _assign(self, name, value):
        a = getattr(self, name)
        v = np.asarray(value, dtype=np.float64)
        if self.nchains == 1:
            a[0] = v
        else:
            a[...] = v

    _b = property(lambda self: self._view(self._b_all),
                  lambda self, v: self._assign("_b_all", v))
    _z = property(lambda self: self._view(self._z_all),
                  lambda self, v: self._assign("_z_all", v))
    _alpha = property(lambda self: self._view(self._alpha_all),
                      lambda self, v: self._assign("_alpha_all", v))
    _pout = property(lambda self: self._view(self._pout_all),
                     lambda self, v: self._assign("_pout_all", v))
    _theta = property(lambda self: self._theta_all[0] if self.nchains == 1 else self._theta_all,
                      lambda self, v: self._assign("_theta_all", v))
    tdf = property(lambda self: self._tdf_all[0] if self.nchains == 1 else self._tdf_all,
                   lambda self, v: self._assign("_tdf_all", v))

    # ---- parameter helpers (gibbs.py:53-77) ----------------------------------------------
    @property
    def params(self):
        return list(self.pta.params)

    def map_params(self, xs):
        return {par.name: x for par, x in zip(self.params, xs)}

    def get_hyper_param_indices(self):
        return np.array([i for i, p in enumerate(self.params)
                         if "ecorr" in p.name or "log10_A" in p.name or "gamma" in p.name])

    def get_white_noise_indices(self):
        return np.array([i for i, p in enumerate(self.params)
                         if "efac" in p.name or "equad" in p.name])

    # ---- likelihoods ----------------------------------------------------------------------
    def get_lnprior(self, xs):
        """gibbs.py:337-339."""
        return sum(p.get_logpdf(x) for p, x in zip(self.params, xs))

    def get_lnlikelihood_df(self, df):
        """gibbs.py:331-335 (host: a 30-point scalar function); one value per chain."""
        n = len(self._residuals)
        a = self._alpha_all
        v = -(df / 2) * np.sum(np.log(a) + 1 / a, axis=1) + n * (df / 2) * np.log(df / 2) \
            - n * scipy.special.gammaln(df / 2)
        return v[0] if self.nchains == 1 else v

    def _xs_all(self, xs):
        xs = np.asarray(xs, dtype=np.float64)
        if xs.ndim == 1:
            xs = np.broadcast_to(xs, (self.nchains, xs.shape[0]))
        return np.ascontiguousarray(xs)

    def _push(self, xs_all):
        self._native.set_state(x=xs_all, b=self._b_all, z=self._z_all, alpha=self._alpha_all,
                               pout=self._pout_all, theta=self._theta_all, nu=self._tdf_all)

    def _pull(self):
        s = self._native.get_state()
        self._b_all, self._z_all, self._alpha_all = s["b"], s["z"], s["alpha"]
        self._pout_all, self._theta_all, self._tdf_all = s["pout"], s["theta"], s["nu"]
        self._x_all = s["x"]
        self.status = s["status"]
        return s["x"]

    def _lnlikes(self, xs):
        self._push(self._xs_all(xs))
        w, h = self._native.eval_lnlike()
        return (w[0], h[0]) if self.nchains == 1 else (w, h)

    def get_lnlikelihood_white(self, xs):
        """gibbs.py:262-284, evaluated on the GPU."""
        return self._lnlikes(xs)[0]

    def get_lnlikelihood(self, xs):
        """gibbs.py:288-329, evaluated on the GPU (Gram + Cholesky)."""
        return self._lnlikes(xs)[1]

    # ---- single-stage updates (each one GPU launch with a stage mask) -----------------------
    # As in the reference (gibbs.py:80-259) a stage method RETURNS its draw and leaves the
    # latent state (_b, _theta, _z, _alpha, tdf) alone; only update_z records _pout
    # (gibbs.py:225).  Callers commit, e.g. ``g._b = g.update_b(x)`` (gibbs.py:374-380).
    # Each call advances the Philox sweep counter, so repeated calls draw afresh.
    def _stage(self, xs, mask):
        self._push(self._xs_all(xs))
        self._native.sweep(1, mask=mask, seed=self.seed, sweep0=self._sweep_counter)
        self._sweep_counter += 1
        s = self._native.get_state()
        self.status = s["status"]
        return s

    def _ret(self, a):
        return a[0] if self.nchains == 1 else a

    def update_white_params(self, xs):
        return self._ret(self._stage(xs, _abi.STAGE_WHITE)["x"])

    def update_hyper_params(self, xs):
        return self._ret(self._stage(xs, _abi.STAGE_HYPER)["x"])

    def update_b(self, xs):
        # a direct call draws unconditionally (gibbs.py:145-182); the :373 test belongs to
        # sample() only
        return self._ret(self._stage(xs, _abi.STAGE_B | _abi.STAGE_B_FORCE)["b"])

    def update_theta(self, xs):
        return self._ret(self._stage(xs, _abi.STAGE_THETA)["theta"])

    def update_z(self, xs):
        s = self._stage(xs, _abi.STAGE_Z)
        if self._lmodel in ("mixture", "vvh17"):
            self._pout_all = s["pout"]                       # gibbs.py:225
        return self._ret(s["z"])

    def update_alpha(self, xs):
        return self._ret(self._stage(xs, _abi.STAGE_ALPHA)["alpha"])

    def update_df(self, xs):
        return self._ret(self._stage(xs, _abi.STAGE_DF)["nu"])

    # ---- the sampler (gibbs.py:342-385) ----------------------------------------------------
    def sample(self, xs, niter=10000):
        C, P = self.nchains, len(self.params)
        n, mcols = len(self._residuals), self._b_all.shape[1]
        every = max(1, self.record_every)
        nrec = (niter + every - 1) // every
        lead = () if C == 1 else (C,)
        self.chain = np.zeros(lead + (nrec, P))
        self.bchain = np.zeros(lead + (nrec, mcols))
        self.thetachain = np.zeros(lead + (nrec,))
        self.zchain = np.zeros(lead + (nrec, n))
        self.alphachain = np.zeros(lead + (nrec, n))
        self.poutchain = np.zeros(lead + (nrec, n))
        self.dfchain = np.zeros(lead + (nrec,))
        outs = {"x": self.chain, "b": self.bchain, "theta": self.thetachain,
                "z": self.zchain, "alpha": self.alphachain, "pout": self.poutchain,
                "nu": self.dfchain}
        self._push(self._xs_all(xs))
        chunk = max(every, (self.chunk // every) * every)
        tstart = time.time()
        done, ri = 0, 0
        while done < niter:
            k = min(chunk, niter - done)
            kr = (k + every - 1) // every
            recs = self._native.alloc_records(kr)
            self._native.sweep(k, records=recs, record_every=every, seed=self.seed,
                               sweep0=self._sweep_counter)
            self._sweep_counter += k
            for key in STATE_KEYS:
                host = recs[key].cpu().numpy()
                if C == 1:
                    outs[key][ri:ri + kr] = host[0]
                else:
                    outs[key][:, ri:ri + kr] = host
            done += k
            ri += kr
            if self.verbose:
                sys.stdout.write("\r")
                sys.stdout.write("Finished %g percent in %g seconds." %
                                 (done / niter * 100, time.time() - tstart))
                sys.stdout.flush()
        x = self._pull()
        self._counter_at_sample = self._sweep_counter
        return x[0] if C == 1 else x

    # ---- checkpoint / resume (not in the reference: gibbs.py:344-350 restarts its chains) --
    def checkpoint(self):
        """The sampler's whole state after ``sample``: every chain's x and latents (b, z,
        alpha, pout, theta, nu), the Philox key and sweep counter, the model options and the
        basis shape.  A sampler restored from it continues the chains bitwise: the kernels
        keep no state across launches, and the variates of a sweep are keyed
        by (seed, sweep index, chain)."""
        if self._x_all is None:
            raise RuntimeError("checkpoint() needs a finished sample() call")
        if self._sweep_counter != self._counter_at_sample:
            # a stage method advanced the Philox counter after sample() returned, so the x
            # of that sample() no longer pairs with the counter: a resume from it would not
            # be the uninterrupted chain
            raise RuntimeError("checkpoint() must directly follow sample(): "
                               f"{self._sweep_counter - self._counter_at_sample} stage "
                               "call(s) ran since")
        return make_checkpoint(self._cfg, self.pta.get_basis()[0].shape, self.seed,
                               self._sweep_counter, fingerprint=dataset_fingerprint(self.pta),
                               x=self._x_all, b=self._b_all,
                               z=self._z_all, alpha=self._alpha_all, pout=self._pout_all,
                               theta=self._theta_all, nu=self._tdf_all)

    def save_checkpoint(self, path):
        """``checkpoint()`` as an .npz file (plain arrays, no pickles)."""
        np.savez(path, **self.checkpoint())

    def load_checkpoint(self, ckpt):
        """Restore a ``checkpoint()`` (dict or .npz path) into this sampler, which must have
        the same model options, basis shape and chain count; returns x to pass to
        ``sample`` (the chains then continue where the checkpointed ones stopped)."""
        if not isinstance(ckpt, dict):
            with np.load(ckpt, allow_pickle=False) as f:
                ckpt = {k: f[k] for k in f.files}
        check_checkpoint(ckpt, self._cfg, self.pta.get_basis()[0].shape, self.nchains,
                         fingerprint=dataset_fingerprint(self.pta))
        self.seed = int(ckpt["seed"])
        self._sweep_counter = int(ckpt["sweep_counter"])
        self._b_all = np.array(ckpt["b"], dtype=np.float64)
        self._z_all = np.array(ckpt["z"], dtype=np.float64)
        self._alpha_all = np.array(ckpt["alpha"], dtype=np.float64)
        self._pout_all = np.array(ckpt["pout"], dtype=np.float64)
        self._theta_all = np.array(ckpt["theta"], dtype=np.float64)
        self._tdf_all = np.array(ckpt["nu"], dtype=np.float64)
        self._x_all = np.array(ckpt["x"], dtype=np.float64)
        self._counter_at_sample = self._sweep_counter
        return self._x_all[0] if self.nchains == 1 else self._x_all

    def close(self):
        self._native.close()


CKPT_VERSION = 2
_CKPT_OPTS = ("model", "tdf", "m", "vary_df", "theta_prior", "vary_alpha", "alpha", "pspin",
              "exact_bdraw")
_CKPT_STR_OPTS = ("model", "theta_prior")


def dataset_fingerprint(pta):
    """SHA-256 of the data a chain's posterior depends on: residuals, error bars, the basis T
    and its Fourier frequencies, the timing-model prior, the backend / ECORR assignment.  A
    checkpoint resumes only on the dataset it was taken on."""
    import hashlib
    h = hashlib.sha256()
    parts = [pta.get_residuals()[0], getattr(pta, "_toaerrs", np.zeros(0)),
             pta.get_basis()[0], getattr(pta, "Ffreqs", np.zeros(0)),
             np.array([float(getattr(pta, "tm_weight", 0.0))]),
             getattr(pta, "bidx", np.zeros(0)), getattr(pta, "ecorr_backend", np.zeros(0))]
    for a in parts:
        a = np.ascontiguousarray(np.asarray(a, dtype=np.float64))
        h.update(str(a.shape).encode())
        h.update(a.tobytes())
    return h.hexdigest()


def _norm_opt(key, v):
    """Option value in a comparable form: tdf = 4 and 4.0, or np.float64(0.01) and 0.01,
    are the same option."""
    if v is None:
        return None
    if key in _CKPT_STR_OPTS:
        return str(v)
    if isinstance(v, (bool, np.bool_)):
        return bool(v)
    return float(v)


def _opts_json(cfg):
    import json
    return json.dumps({k: _norm_opt(k, cfg.get(k)) for k in _CKPT_OPTS}, sort_keys=True)


def make_checkpoint(cfg, basis_shape, seed, sweep_counter, fingerprint="", **state):
    """Checkpoint dict: state arrays (leading chain axis) + key, counter, options (JSON of
    normalised values), basis shape and the dataset fingerprint."""
    ck = {k: np.asarray(v, dtype=np.float64) for k, v in state.items()}
    ck.update(version=np.int64(CKPT_VERSION), seed=np.uint64(seed),
              sweep_counter=np.int64(sweep_counter), n=np.int64(basis_shape[0]),
              m=np.int64(basis_shape[1]), options=np.array(_opts_json(cfg)),
              fingerprint=np.array(str(fingerprint)))
    return ck


def check_checkpoint(ck, cfg, basis_shape, nchains, fingerprint=None):
    """Raise ValueError unless ``ck`` fits a sampler with these options / shape / chains (and,
    when ``fingerprint`` is given, was taken on the same dataset)."""
    import json
    if int(ck.get("version", -1)) != CKPT_VERSION:
        raise ValueError(f"checkpoint version {ck.get('version')} != {CKPT_VERSION}")
    got = json.loads(str(np.asarray(ck["options"])))
    want = json.loads(_opts_json(cfg))
    if got != want:
        diff = {k: (got.get(k), want.get(k)) for k in want if got.get(k) != want.get(k)}
        raise ValueError(f"checkpoint model options differ (checkpoint, sampler): {diff}")
    if (int(ck["n"]), int(ck["m"])) != tuple(basis_shape):
        raise ValueError(f"checkpoint basis {int(ck['n'])}x{int(ck['m'])} != "
                         f"{basis_shape[0]}x{basis_shape[1]}")
    if fingerprint is not None and str(np.asarray(ck["fingerprint"])) != str(fingerprint):
        raise ValueError("checkpoint was taken on a different dataset (residuals, error bars "
                         "or basis differ)")
    for k in ("x", "b", "z", "alpha", "pout", "theta", "nu"):
        if np.asarray(ck[k]).shape[0] != nchains:
            raise ValueError(f"checkpoint has {np.asarray(ck[k]).shape[0]} chains, "
                             f"sampler {nchains}")
