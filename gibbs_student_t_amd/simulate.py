"""Batched synthetic pulsars on the GPU: the simulate_data.py:10-39 recipe (gst_simulate).

The reference makes one fake pulsar per call through libstempo (log-normal error bars,
power-law red noise, Bernoulli(theta) outliers, a refit, then the no_outlier copy with the
outlier TOAs deleted, simulate_data.py:12-37) and run_sims.py:41-51 re-reads both from
par/tim.  Here one launch draws D datasets at given epochs (one workgroup per dataset,
Philox keyed by (seed, dataset0 + d), so shards of a grid draw the same datasets), and
``pairs`` turns them into the (outlier, no_outlier) PulsarData the sampler takes.  The
CPU restatement that pins the kernel is oracle/sim_oracle.py.
"""
from __future__ import annotations

import ctypes as ct

import numpy as np

from . import _abi
from .model import FYR, PulsarData, fourier_basis, svd_tm_basis


def _per_dataset(v, D, name):
    a = np.broadcast_to(np.asarray(v, dtype=np.float64), (D,)).copy()
    if not np.all(np.isfinite(a)):
        raise ValueError(f"{name} must be finite")
    return a


def simulate_batch(toas, Mmat, n_datasets: int, *, seed: int, dataset0: int = 0,
                   theta=0.05, sigma_out=1e-6, log10_A=-14.0, gamma=4.33, dof=None,
                   components: int = 30, red=None, toaerrs=None, clean: bool = True,
                   device: int = 0, Tspan=None):
    """Draw ``n_datasets`` pulsars at the epochs ``toas`` (s) with timing model ``Mmat``.

    Per-dataset parameters (theta, sigma_out, log10_A, gamma, dof) are scalars or length-D
    arrays; ``dof`` None / <= 0 is Gaussian white noise.  ``red`` (n values, s) replaces the
    power-law draw (red.txt); ``toaerrs`` (n, s) replaces the log-normal error
    bars.  Returns numpy arrays ``residuals``, ``toaerrs``, ``z`` [D, n] and, with ``clean``,
    ``residuals_clean`` [D, n] (the no_outlier twin's refit residuals; 0 at outliers)."""
    import torch
    toas = np.asarray(toas, dtype=np.float64)
    n = len(toas)
    D = int(n_datasets)
    U = svd_tm_basis(np.asarray(Mmat, dtype=np.float64))[0]
    F, ff = fourier_basis(toas, components, Tspan)
    f = ff[::2]
    df = np.diff(np.concatenate(([0.0], f)))
    dev = torch.device("cuda", device)

    def put(a):
        return None if a is None else torch.as_tensor(
            np.ascontiguousarray(a, dtype=np.float64)).to(dev)

    keep = []

    def ptr(t):
        if t is None:
            return None
        keep.append(t)
        return ct.c_void_p(t.data_ptr())

    dofs = np.zeros(D) if dof is None else _per_dataset(dof, D, "dof")
    f64 = dict(dtype=torch.float64, device=dev)
    out = {"residuals": torch.empty((D, n), **f64), "toaerrs": torch.empty((D, n), **f64),
           "z": torch.empty((D, n), **f64)}
    if clean:
        out["residuals_clean"] = torch.empty((D, n), **f64)
    desc = _abi.SimDesc(
        n=n, nfourier=2 * components, ntm=U.shape[1], ndatasets=D,
        F=ptr(put(F)), log_f=ptr(put(np.log(ff))), log_df=ptr(put(np.log(np.repeat(df, 2)))),
        log_fyr=float(np.log(FYR)), U=ptr(put(U)),
        red=ptr(put(None if red is None else np.asarray(red, dtype=np.float64))),
        toaerrs=ptr(put(None if toaerrs is None else np.asarray(toaerrs, dtype=np.float64))),
        theta=ptr(put(_per_dataset(theta, D, "theta"))),
        sigma_out=ptr(put(_per_dataset(sigma_out, D, "sigma_out"))),
        log10_A=ptr(put(_per_dataset(log10_A, D, "log10_A"))),
        gamma=ptr(put(_per_dataset(gamma, D, "gamma"))), dof=ptr(put(dofs)),
        seed=int(seed) & 0xFFFFFFFFFFFFFFFF, dataset0=int(dataset0),
        residuals=ptr(out["residuals"]), toaerrs_out=ptr(out["toaerrs"]), z=ptr(out["z"]),
        residuals_clean=ptr(out.get("residuals_clean")))
    lib = _abi.load()
    with torch.cuda.device(dev):
        stream = torch.cuda.current_stream(dev).cuda_stream
        _abi.check(lib, lib.gst_simulate(ct.byref(desc), ct.c_void_p(stream)), "gst_simulate")
        torch.cuda.synchronize(dev)
    res = {k: v.cpu().numpy() for k, v in out.items()}
    res["z"] = res["z"].astype(np.int64)
    return res


def pairs(toas, Mmat, sim, name: str = "PSR", freqs=None):
    """The (outlier, no_outlier) PulsarData of every simulated dataset, as
    simulate_data.py:28-37 writes them: the no_outlier pulsar keeps only the z == 0 TOAs
    (and their timing-model rows), with the residuals refit on them."""
    toas = np.asarray(toas, dtype=np.float64)
    Mmat = np.asarray(Mmat, dtype=np.float64)
    out = []
    for d in range(sim["residuals"].shape[0]):
        z = sim["z"][d]
        a = PulsarData(name=name, toas=toas, residuals=sim["residuals"][d],
                       toaerrs=sim["toaerrs"][d], Mmat=Mmat, freqs=freqs,
                       meta={"z_true": z, "dataset": d})
        b = None
        if "residuals_clean" in sim:
            k = z == 0
            b = PulsarData(name=name, toas=toas[k], residuals=sim["residuals_clean"][d][k],
                           toaerrs=sim["toaerrs"][d][k], Mmat=Mmat[k],
                           freqs=None if freqs is None else np.asarray(freqs)[k],
                           meta={"dataset": d})
        out.append((a, b))
    return out


__all__ = ["simulate_batch", "pairs"]
