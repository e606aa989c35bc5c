"""Structured single-pulsar noise model: the "pta" object `Gibbs` consumes.

The reference sampler (`/root/reference/gibbs.py`) talks to an enterprise ``PTA``
through five duck-typed calls:

* ``get_residuals()[0]``                       (gibbs.py:29)
* ``get_basis(params)[0]``                     (gibbs.py:35,158,210,236,269,301)
* ``get_ndiag(params)[0]``                     (gibbs.py:154,209,235,268,297)
* ``get_phiinv(params, logdet=...)[0]``        (gibbs.py:155,298)
* ``params`` (objects with ``.name``, ``.get_logpdf``, ``.sample``)  (gibbs.py:56,339;
  run_sims.py:111)

enterprise is not installed here (no network) and is not vendored by the reference, so
this module restates the *specific* model `run_sims.py:57-83` builds:

* white noise ``N0 = efac^2 * sigma^2 + 10^(2*log10_equad)``  (MeasurementNoise + EquadNoise,
  run_sims.py:57-62); efac is ``Constant(1.0)`` there, ``Uniform(0.2, 10)`` in the notebook.
* red noise: Fourier GP, ``components`` sin/cos pairs on ``f_k = k / Tspan``, power-law
  spectrum with ``log10_A ~ U(-18,-12)``, ``gamma ~ U(1,7)`` (run_sims.py:65-66).
* timing model: ``BasisGP`` on the SVD basis ``U`` of the design matrix with prior weight
  ``1e40`` (run_sims.py:22-29,69-71).

and, as the notebook's J1643-1224 model uses them (gibbs_likelihood.ipynb cell 2), the
general white-noise options the reference sampler handles through its index sets
(gibbs.py:64-77: any ``ecorr`` parameter is a hyper parameter, any ``efac``/``equad`` a white
one):

* ``selection="backend"``: one efac / log10_equad (/ log10_ecorr) per backend
  (enterprise ``selections.by_backend``), parameters named ``{psr}_{backend}_efac`` etc.;
  ``"none"`` (``no_selection``): one set named ``{psr}_efac`` etc.
* ``log10_ecorr=(pmin, pmax)``: ECORR as a basis GP (enterprise ``EcorrBasisModel``): one
  column per observing epoch with at least two TOAs (``quantization_matrix``), per backend
  under ``selection="backend"``, prior variance ``10^(2 log10_ecorr)``.

The enterprise formulas (Fourier design matrix, power law, ``phiinv``/``logdet`` from a
diagonal ``phi``) are restated from their published form; parity against enterprise
itself is **unpinned** (no fixture of it exists in the reference).  Everything else in the
build -- the CPU oracle, the golden generator and the HIP path -- consumes this one model,
so the sampler parity is exact with respect to it.

Column order of the basis ``T`` is ``[Fourier (2*components) | timing model | ECORR]`` as in
enterprise's signal-collection order ``ef + eq + rn + tm (+ ec)`` (run_sims.py:74,
gibbs_likelihood.ipynb cell 2).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

# enterprise.constants: yr = 365.25 * 86400 s, fyr = 1 / yr
YR_SEC = 365.25 * 86400.0
FYR = 1.0 / YR_SEC
DAY_SEC = 86400.0


class Constant:
    """A fixed parameter (enterprise ``parameter.Constant``); never sampled."""

    def __init__(self, value: float):
        self.value = float(value)


class Uniform:
    """Uniform prior parameter (enterprise ``parameter.Uniform``).

    ``get_logpdf`` is ``scipy.stats.uniform(pmin, pmax - pmin).logpdf``: ``-log(pmax-pmin)``
    on the closed interval, ``-inf`` outside (called at gibbs.py:339).
    """

    def __init__(self, name: str, pmin: float, pmax: float):
        self.name = name
        self.pmin = float(pmin)
        self.pmax = float(pmax)
        self.logpdf_in = -np.log(self.pmax - self.pmin)

    def get_logpdf(self, value):
        value = float(value)
        if self.pmin <= value <= self.pmax:
            return self.logpdf_in
        return -np.inf

    def sample(self):
        # run_sims.py:111 draws the initial point from the priors
        return np.random.uniform(self.pmin, self.pmax)

    def __repr__(self):
        return f"{self.name}:Uniform(pmin={self.pmin}, pmax={self.pmax})"


def fourier_basis(toas: np.ndarray, nmodes: int, Tspan: float | None = None):
    """Red-noise Fourier design matrix (enterprise ``createfourierdesignmatrix_red``).

    Columns alternate sin/cos of ``2 pi f_k t`` with ``f_k = k / Tspan``, k = 1..nmodes.
    Returns ``(F, Ffreqs)`` with ``Ffreqs = repeat(f, 2)``.
    """
    T = Tspan if Tspan is not None else toas.max() - toas.min()
    f = np.linspace(1.0 / T, nmodes / T, nmodes)
    F = np.zeros((len(toas), 2 * nmodes))
    arg = 2.0 * np.pi * toas[:, None] * f[None, :]
    F[:, ::2] = np.sin(arg)
    F[:, 1::2] = np.cos(arg)
    return F, np.repeat(f, 2)


def powerlaw(f: np.ndarray, log10_A: float, gamma: float, components: int = 2):
    """Power-law prior variances (enterprise ``utils.powerlaw``).

    ``phi_k = A^2 / 12 / pi^2 * fyr^(gamma-3) * f_k^(-gamma) * df_k``.  The left-to-right
    evaluation order is part of the contract the HIP kernel reproduces.
    """
    df = np.diff(np.concatenate((np.array([0.0]), f[::components])))
    return ((10 ** log10_A) ** 2 / 12.0 / np.pi ** 2 * FYR ** (gamma - 3)
            * f ** (-gamma) * np.repeat(df, components))


def quantization_matrix(toas: np.ndarray, dt: float = 1.0, nmin: int = 2):
    """Epoch basis of ECORR (enterprise ``utils.create_quantization_matrix``): TOAs sorted
    by time, a new epoch whenever a TOA is ``dt`` seconds or more after the epoch's first
    TOA; epochs with fewer than ``nmin`` TOAs get no column.  Returns ``U`` (n x epochs,
    one 1 per row of a TOA in a kept epoch)."""
    toas = np.asarray(toas, dtype=np.float64)
    isort = np.argsort(toas, kind="stable")
    buckets = [[isort[0]]] if len(toas) else []
    ref = toas[isort[0]] if len(toas) else 0.0
    for i in isort[1:]:
        if toas[i] - ref < dt:
            buckets[-1].append(i)
        else:
            buckets.append([i])
            ref = toas[i]
    buckets = [b for b in buckets if len(b) >= nmin]
    U = np.zeros((len(toas), len(buckets)))
    for e, b in enumerate(buckets):
        U[b, e] = 1.0
    return U


def svd_tm_basis(Mmat: np.ndarray):
    """Timing-model basis: left singular vectors of the design matrix (run_sims.py:22-25)."""
    u, s, _ = np.linalg.svd(Mmat, full_matrices=False)
    return u, np.ones_like(s)


@dataclass
class PulsarData:
    """What the sampler needs from a pulsar (enterprise ``Pulsar`` subset)."""

    name: str
    toas: np.ndarray        # seconds
    residuals: np.ndarray   # seconds
    toaerrs: np.ndarray     # seconds
    Mmat: np.ndarray        # timing-model design matrix (n x ntm)
    freqs: np.ndarray | None = None
    meta: dict = field(default_factory=dict)
    backends: np.ndarray | None = None   # backend label of each TOA (tim-file flag -be/-f)

    @property
    def n(self):
        return len(self.toas)


class PTA:
    """Single-pulsar model with the enterprise ``PTA`` protocol used by ``Gibbs``.

    Parameters mirror run_sims.py:57-71.  ``efac`` may be a float (constant, run_sims)
    or a ``(pmin, pmax)`` tuple (varied, as in the notebook).
    """

    def __init__(self, psr: PulsarData, components: int = 30, efac=1.0,
                 log10_equad=(-10.0, -5.0), log10_A=(-18.0, -12.0), gamma=(1.0, 7.0),
                 tm_weight: float = 1e40, Tspan: float | None = None, *,
                 selection: str = "none", log10_ecorr=None, ecorr_dt: float = 1.0):
        self.psr = psr
        self.components = int(components)
        self._r = np.asarray(psr.residuals, dtype=np.float64)
        self._toaerrs = np.asarray(psr.toaerrs, dtype=np.float64)
        toas = np.asarray(psr.toas, dtype=np.float64)
        self.F, self.Ffreqs = fourier_basis(toas, self.components, Tspan)
        U, w = svd_tm_basis(np.asarray(psr.Mmat, dtype=np.float64))
        self.U = U
        self.tm_phi = w * tm_weight          # tm_prior (run_sims.py:27-29)
        self.tm_weight = float(tm_weight)
        self._set_backends(psr.backends, selection)
        cols, self.ecorr_backend = [], np.zeros(0, dtype=np.int64)
        if log10_ecorr is not None:
            # one quantization per backend (enterprise applies the basis per selection mask)
            eb = []
            for b in range(len(self.backend_names)):
                mask = self.bidx == b
                Ub = quantization_matrix(toas[mask], ecorr_dt)
                full = np.zeros((len(toas), Ub.shape[1]))
                full[mask] = Ub
                cols.append(full)
                eb += [b] * Ub.shape[1]
            self.ecorr_backend = np.array(eb, dtype=np.int64)
        self.Uec = np.hstack(cols) if cols else np.zeros((len(toas), 0))
        self.T = np.hstack([self.F, self.U, self.Uec])
        self._build_params(efac, log10_equad, log10_A, gamma, log10_ecorr)

    # --- white-noise structure ----------------------------------------------------------
    def _set_backends(self, backends, selection):
        if selection not in ("none", "backend"):
            raise ValueError("selection must be 'none' or 'backend'")
        n = len(self._r)
        self.selection = selection
        if selection == "backend":
            if backends is None:
                raise ValueError("selection='backend' needs psr.backends")
            labels = np.asarray(backends).astype(str)
            self.backend_names = sorted(set(labels.tolist()))
            self.bidx = np.array([self.backend_names.index(v) for v in labels], dtype=np.int64)
        else:
            self.backend_names = [""]
            self.bidx = np.zeros(n, dtype=np.int64)

    def _pname(self, b, what):
        be = self.backend_names[b]
        return f"{self.psr.name}_{be}_{what}" if be else f"{self.psr.name}_{what}"

    def _build_params(self, efac, log10_equad, log10_A, gamma, log10_ecorr):
        nm = self.psr.name
        plist = []
        nb = len(self.backend_names)
        if isinstance(efac, (tuple, list)):
            plist += [Uniform(self._pname(b, "efac"), *efac) for b in range(nb)]
            self.efac_const = None
        else:
            self.efac_const = float(efac)
        plist += [Uniform(self._pname(b, "log10_equad"), *log10_equad) for b in range(nb)]
        if log10_ecorr is not None:
            plist += [Uniform(self._pname(b, "log10_ecorr"), *log10_ecorr) for b in range(nb)]
        plist.append(Uniform(f"{nm}_log10_A", *log10_A))
        plist.append(Uniform(f"{nm}_gamma", *gamma))
        # enterprise returns params sorted by name
        self._params = sorted(plist, key=lambda p: p.name)
        self.has_ecorr = log10_ecorr is not None

    @classmethod
    def from_arrays(cls, name, residuals, toaerrs, T, Ffreqs, components, tm_weight=1e40,
                    efac=1.0, **priors):
        """Rebuild a model from stored arrays (golden fixtures) without re-deriving T."""
        obj = cls.__new__(cls)
        obj.psr = PulsarData(name=str(name), toas=np.zeros(len(residuals)),
                             residuals=np.asarray(residuals), toaerrs=np.asarray(toaerrs),
                             Mmat=np.zeros((len(residuals), 0)))
        obj.components = int(components)
        obj._r = np.asarray(residuals, dtype=np.float64)
        obj._toaerrs = np.asarray(toaerrs, dtype=np.float64)
        nf = 2 * obj.components
        T = np.asarray(T, dtype=np.float64)
        obj.F, obj.Ffreqs = T[:, :nf], np.asarray(Ffreqs, dtype=np.float64)
        obj.U = T[:, nf:]
        obj.tm_weight = float(tm_weight)
        n_ec = int(priors.pop("n_ecorr", 0))
        ntm = T.shape[1] - nf - n_ec
        obj.U = T[:, nf:nf + ntm]
        obj.Uec = T[:, nf + ntm:]
        obj.tm_phi = np.ones(obj.U.shape[1]) * obj.tm_weight
        obj.T = T
        obj.psr.backends = priors.pop("backends", None)
        obj._set_backends(obj.psr.backends, priors.pop("selection", "none"))
        eb = priors.pop("ecorr_backend", None)
        obj.ecorr_backend = (np.zeros(0, dtype=np.int64) if eb is None
                             else np.asarray(eb, dtype=np.int64))
        obj._build_params(efac, priors.get("log10_equad", (-10., -5.)),
                          priors.get("log10_A", (-18., -12.)), priors.get("gamma", (1., 7.)),
                          priors.get("log10_ecorr"))
        return obj

    # --- the protocol ---------------------------------------------------------------
    @property
    def params(self):
        return list(self._params)

    @property
    def param_names(self):
        return [p.name for p in self._params]

    def get_residuals(self):
        return [self._r]

    def get_basis(self, params=None):
        return [self.T]

    def _value(self, params, suffix):
        return params[f"{self.psr.name}_{suffix}"]

    def get_ndiag(self, params):
        if len(self.backend_names) == 1:
            efac = (self.efac_const if self.efac_const is not None
                    else params[self._pname(0, "efac")])
            eq = params[self._pname(0, "log10_equad")]
            return [efac ** 2 * self._toaerrs ** 2 + 10 ** (2 * eq) * np.ones(len(self._r))]
        nb = len(self.backend_names)
        efac = np.array([self.efac_const if self.efac_const is not None
                         else params[self._pname(b, "efac")] for b in range(nb)])[self.bidx]
        eq = np.array([params[self._pname(b, "log10_equad")] for b in range(nb)])[self.bidx]
        return [efac ** 2 * self._toaerrs ** 2 + 10 ** (2 * eq)]

    def get_phi(self, params):
        pl = powerlaw(self.Ffreqs, self._value(params, "log10_A"),
                      self._value(params, "gamma"), components=2)
        parts = [pl, self.tm_phi]
        if self.n_ecorr:
            ec = np.array([params[self._pname(b, "log10_ecorr")]
                           for b in range(len(self.backend_names))])
            parts.append(10 ** (2 * ec[self.ecorr_backend]))
        return [np.concatenate(parts)]

    def get_phiinv(self, params, logdet=False):
        phi = self.get_phi(params)[0]
        if logdet:
            return [(1.0 / phi, np.sum(np.log(phi)))]
        return [1.0 / phi]

    # --- convenience for the native path --------------------------------------------
    @property
    def n(self):
        return self.T.shape[0]

    @property
    def m(self):
        return self.T.shape[1]

    @property
    def nfourier(self):
        return 2 * self.components

    @property
    def ntm(self):
        return self.U.shape[1]

    @property
    def n_ecorr(self):
        return self.Uec.shape[1]

    @property
    def nbackend(self):
        return len(self.backend_names)

    def backend_param_indices(self, what):
        """Index into ``params`` of each backend's ``what`` parameter (-1: none / constant)."""
        names = self.param_names
        return np.array([names.index(self._pname(b, what)) if self._pname(b, what) in names
                         else -1 for b in range(len(self.backend_names))], dtype=np.int64)

    def param_index(self, suffix):
        for i, p in enumerate(self._params):
            if p.name.endswith("_" + suffix):
                return i
        return -1

    def sample_params(self):
        return np.array([p.sample() for p in self._params]).flatten()


def df_tables(n: int):
    """Constant parts of the dof log-density (gibbs.py:331-335) for nu = 1..30.

    ``ll(nu) = -(nu/2)*S + A[nu] - B[nu]`` with ``A = n*(nu/2)*log(nu/2)`` and
    ``B = n*gammaln(nu/2)``; evaluated on the host exactly as the reference does so the
    device only adds ``-(nu/2)*S``.
    """
    import scipy.special
    dfs = np.arange(1, 31)
    A = np.array([n * (df / 2) * np.log(df / 2) for df in dfs])
    B = np.array([n * scipy.special.gammaln(df / 2) for df in dfs])
    return A, B


def hyper_white_indices(names):
    """Parameter index sets (gibbs.py:64-77): hyper = ecorr/log10_A/gamma, white = efac/equad."""
    hind = [i for i, nm in enumerate(names)
            if "ecorr" in nm or "log10_A" in nm or "gamma" in nm]
    wind = [i for i, nm in enumerate(names) if "efac" in nm or "equad" in nm]
    return np.array(hind, dtype=np.int64), np.array(wind, dtype=np.int64)


def mh_constants():
    """Jump-scale mixture of the MH proposals (gibbs.py:93-94,126-127)."""
    return np.array([0.1, 0.15, 0.5, 0.15, 0.1]), np.array([0.1, 0.5, 1.0, 3.0, 10.0])


__all__ = ["Constant", "Uniform", "PulsarData", "PTA", "fourier_basis", "powerlaw",
           "svd_tm_basis", "quantization_matrix", "df_tables", "hyper_white_indices", "mh_constants",
           "FYR", "YR_SEC", "DAY_SEC"]
