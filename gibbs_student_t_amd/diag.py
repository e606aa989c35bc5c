"""Convergence diagnostics for batched chains: rank-normalised split-R-hat and bulk-ESS.

The reference has none; the benchmark's ESS/s metric is defined with
these (Vehtari, Gelman, Simpson, Carpenter & Buerkner 2021, "Rank-normalization, folding,
and localization: an improved R-hat").  Inputs are arrays shaped (chains, draws).
"""
from __future__ import annotations

import numpy as np
import scipy.special
import scipy.stats


def _split(x: np.ndarray) -> np.ndarray:
    n = x.shape[1] // 2
    return np.concatenate([x[:, :n], x[:, x.shape[1] - n:]], axis=0)


def _rank_normalise(x: np.ndarray) -> np.ndarray:
    r = scipy.stats.rankdata(x, method="average").reshape(x.shape)
    return scipy.special.ndtri((r - 3.0 / 8.0) / (x.size - 2.0 * 3.0 / 8.0 + 1.0))


def _autocov(x: np.ndarray) -> np.ndarray:
    """Per-chain autocovariance via FFT, biased estimator (as in Stan)."""
    m, n = x.shape
    xc = x - x.mean(axis=1, keepdims=True)
    nfft = 1 << int(np.ceil(np.log2(2 * n)))
    f = np.fft.rfft(xc, n=nfft, axis=1)
    ac = np.fft.irfft(f * np.conj(f), n=nfft, axis=1)[:, :n]
    return ac / n


def ess_raw(x: np.ndarray) -> float:
    """Multi-chain effective sample size (Geyer initial monotone sequence)."""
    x = np.asarray(x, dtype=np.float64)
    m, n = x.shape
    if n < 4:
        return float("nan")
    acov = _autocov(x)
    chain_var = acov[:, 0] * n / (n - 1.0)
    mean_var = chain_var.mean()
    var_plus = mean_var * (n - 1.0) / n
    if m > 1:
        var_plus += x.mean(axis=1).var(ddof=1)
    if not var_plus > 0:
        return float("nan")
    rho = 1.0 - (mean_var - acov.mean(axis=0)) / var_plus
    rho[0] = 1.0
    # Geyer: sum adjacent pairs while positive, enforce monotone decrease
    t = 0
    pairs = []
    while t + 1 < n:
        p = rho[t] + rho[t + 1]
        if p < 0:
            break
        pairs.append(p)
        t += 2
    pairs = np.minimum.accumulate(np.array(pairs)) if pairs else np.array([1.0])
    tau = -1.0 + 2.0 * pairs.sum()
    tau = max(tau, 1.0 / np.log10(m * n))
    return float(m * n / tau)


def bulk_ess(x: np.ndarray) -> float:
    """Rank-normalised split-chain bulk ESS, total over all chains."""
    x = np.asarray(x, dtype=np.float64)
    if np.all(x == x.flat[0]):
        return float("nan")
    return ess_raw(_rank_normalise(_split(x)))


def split_rhat(x: np.ndarray) -> float:
    """Rank-normalised split-R-hat (max of bulk and folded-tail versions)."""
    x = np.asarray(x, dtype=np.float64)

    def _rhat(y):
        m, n = y.shape
        w = y.var(axis=1, ddof=1).mean()
        b = n * y.mean(axis=1).var(ddof=1)
        if not w > 0:
            return float("nan")
        return float(np.sqrt(((n - 1) / n * w + b / n) / w))

    s = _split(x)
    bulk = _rhat(_rank_normalise(s))
    fold = _rhat(_rank_normalise(np.abs(s - np.median(s))))
    return max(bulk, fold)


def ess_rhat(x: np.ndarray):
    """(bulk_ess(x), split_rhat(x)) sharing one rank normalisation of the split chains
    (the costly step at thousands of chains)."""
    x = np.asarray(x, dtype=np.float64)
    if np.all(x == x.flat[0]):
        return float("nan"), float("nan")
    s = _split(x)
    z = _rank_normalise(s)

    def _rhat(y):
        m, n = y.shape
        w = y.var(axis=1, ddof=1).mean()
        b = n * y.mean(axis=1).var(ddof=1)
        if not w > 0:
            return float("nan")
        return float(np.sqrt(((n - 1) / n * w + b / n) / w))

    fold = _rhat(_rank_normalise(np.abs(s - np.median(s))))
    return ess_raw(z), max(_rhat(z), fold)


def ar1_ess(rho: float, m: int, n: int) -> float:
    """Closed-form ESS of m AR(1) chains of length n with coefficient rho (test oracle)."""
    return m * n * (1.0 - rho) / (1.0 + rho)


def summarise(chains: dict) -> dict:
    """{name: (chains, draws) array} -> {name: {"ess": ..., "rhat": ...}}."""
    return {k: {"ess": bulk_ess(v), "rhat": split_rhat(v)} for k, v in chains.items()}
