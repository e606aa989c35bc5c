"""Where does the ``ecq`` theta gap come from?  

The GPU's theta posterior mean on ``ecq`` sits below the reference's long runs.  Two things
separate the GPU chain from the reference chain besides the kernel code itself:

* the **samplers**: the kernel draws Gamma by Marsaglia-Tsang with the a+1 boost for a < 1
  (``gst_kernel.hpp`` gamma_mt), the theta Beta as Ga / (Ga + Gb), normals by Box-Muller;
  the reference uses numpy's legacy samplers (``scipy.stats.gamma/beta.rvs``,
  ``np.random.randn``; gibbs.py:97,130,180,196,239);
* the **b draw**: the kernel draws b exactly (Cholesky, plus the SVD-floor rule where
  Sigma is beyond fp64's resolution); the reference maps normals through ``sl.svd(Sigma)``
  (gibbs.py:169-180), whose small singular values LAPACK resolves only to ~eps * s_max.

This runs the oracle (the reference algorithm, oracle/gibbs_oracle.py) on a 2 x 2 grid --
{numpy legacy samplers, the kernel's samplers on numpy uniforms} x {SVD b draw, the kernel's
exact / floor b draw} -- for C chains x S sweeps each from prior draws, and reports theta's
posterior mean with a chain-means standard error.  Test infrastructure (tools/), never
shipped.

    python tools/ecq_theta_bias.py SWEEPS CHAINS [dataset] [variants]
        variants: comma list of numpy-svd, numpy-floor, kernel-svd, kernel-floor
"""
from __future__ import annotations

import json
import math
import os
import subprocess
import sys
import time
import warnings

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
BURN, THIN = 1000, 5


class KernelSamplerVariates:
    """The HIP kernel's samplers on numpy uniforms (distributionally the kernel's; the
    uniform stream is numpy's, not Philox).

    * MH scale / index / accept: one uniform each through the reference's inverse maps
      (gst_kernel.hpp: choice_from_uniform, gibbs.py:95-104);
    * jumps and b normals: Box-Muller on (1 - u1, u2) (normal_pair);
    * Gamma(a): Marsaglia-Tsang, a < 1 via Gamma(a + 1) * (1 - u)^(1/a), attempts in pairs
      sharing one Box-Muller draw (gamma_mt);
    * Beta(a, b) = Ga / (Ga + Gb) (the theta stage, gst_kernel.hpp:2362-2369);
    * Bernoulli: numpy's legacy inversion on one uniform (bern_legacy);
    * nu: choice on one uniform.
    """

    def __init__(self, seed):
        self.g = np.random.default_rng(seed)

    def _u(self, k=None):
        return self.g.random(k)

    def _normals(self, k):
        h = (k + 1) // 2
        a, b = self._u(h), self._u(h)
        r = np.sqrt(-2.0 * np.log(1.0 - a))
        # normals 2l, 2l + 1 from draw l (normal_pair)
        return np.ravel(np.column_stack([r * np.cos(2 * np.pi * b),
                                         r * np.sin(2 * np.pi * b)]))[:k]

    def scale(self, stage, step):
        from oracle.gibbs_oracle import MH_PROBS, MH_SIZES, choice_from_uniform
        return choice_from_uniform(MH_SIZES, MH_PROBS, self._u())

    def index(self, stage, step, ind):
        ind = np.asarray(ind)
        if len(ind) == 1:
            return ind[:1]
        return np.array([ind[min(int(self._u() * len(ind)), len(ind) - 1)]])

    def jump(self, stage, step, k):
        return self._normals(k)

    def accept_u(self, stage, step):
        return self._u()

    def b_normals(self, m):
        return self._normals(m)

    def gamma(self, shape):
        return gamma_mt_vec(np.atleast_1d(np.asarray(shape, dtype=np.float64)), self._u)

    def beta(self, a, b):
        g = gamma_mt_vec(np.array([a, b], dtype=np.float64), self._u)
        return float(g[0] / (g[0] + g[1]))

    def bernoulli(self, q):
        from oracle.gibbs_oracle import bernoulli_from_uniform
        u = self._u(len(q))
        return np.array([bernoulli_from_uniform(min(qi, 1.0), ui) for qi, ui in zip(q, u)])

    def df_choice(self, p):
        from oracle.gibbs_oracle import DF_GRID, choice_from_uniform
        return choice_from_uniform(DF_GRID, p, self._u())


def gamma_mt_vec(a, unif):
    """gamma_mt (gst_kernel.hpp:479-510) for an array of shapes, vectorised over draws."""
    a = np.array(a, dtype=np.float64)
    out = np.empty_like(a)
    boost = np.ones_like(a)
    small = a < 1.0
    if small.any():
        ub = unif(int(small.sum()))
        boost[small] = np.exp(np.log(1.0 - ub) / a[small])
        a[small] += 1.0
    d = a - 1.0 / 3.0
    cc = 1.0 / np.sqrt(9.0 * d)
    pend = np.arange(len(a))
    for _ in range(128):
        if len(pend) == 0:
            break
        k = len(pend)
        u1, u2, ua, ub = unif(k), unif(k), unif(k), unif(k)
        r = np.sqrt(-2.0 * np.log(1.0 - u1))
        done = np.zeros(k, dtype=bool)
        for h in range(2):
            xn = r * (np.cos(2 * np.pi * u2) if h == 0 else np.sin(2 * np.pi * u2))
            u3 = ua if h == 0 else ub
            dd, c = d[pend], cc[pend]
            v = 1.0 + c * xn
            ok = (v > 0.0) & ~done
            v3 = np.where(ok, v, 1.0) ** 3
            x2 = xn * xn
            with np.errstate(divide="ignore", invalid="ignore"):
                acc = ok & ((u3 < 1.0 - 0.0331 * x2 * x2) |
                            (np.log(u3) < 0.5 * x2 + dd * (1.0 - v3 + np.log(v3))))
            idx = pend[acc]
            out[idx] = dd[acc] * v3[acc] * boost[idx]
            done |= acc
        pend = pend[~done]
    if len(pend):
        out[pend] = d[pend] * boost[pend]
    return out


def worker(dataset, model, variant, sweeps, seed, path):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    warnings.filterwarnings("ignore")
    from golden_io import load_dataset
    from gibbs_student_t_amd.run_sims import MODELS
    from oracle.gibbs_oracle import LegacyNumpyVariates, Oracle, OutlierModel, initial_state
    pta = load_dataset(dataset=dataset)
    np.random.seed(seed)
    x = np.array(pta.sample_params(), dtype=np.float64)
    samp, bdraw = variant.split("-")
    src = LegacyNumpyVariates() if samp == "numpy" else KernelSamplerVariates(seed)
    orc = Oracle(pta, OutlierModel(**MODELS[model]))
    st = initial_state(pta, orc.cfg)
    th, nu, xs = [], [], []
    t0 = time.time()
    for i in range(sweeps):
        if i >= BURN and (i - BURN) % THIN == 0:
            th.append(st.theta)
            nu.append(float(st.nu))
            xs.append(x.copy())
        x = orc.sweep(st, x, src, b_mean="svd" if bdraw == "svd" else "floor")
    np.savez(path, theta=np.array(th), nu=np.array(nu), x=np.array(xs),
             secs=time.time() - t0)


def main():
    if sys.argv[1:2] == ["--worker"]:
        a = sys.argv[2:]
        worker(a[0], a[1], a[2], int(a[3]), int(a[4]), a[5])
        return
    sweeps = int(sys.argv[1])
    chains = int(sys.argv[2])
    dataset = sys.argv[3] if len(sys.argv) > 3 else "ecq"
    variants = (sys.argv[4] if len(sys.argv) > 4 else
                "numpy-svd,numpy-floor,kernel-svd,kernel-floor").split(",")
    nproc = int(os.environ.get("NPROC", "8"))
    env = dict(os.environ, OPENBLAS_NUM_THREADS="1", OMP_NUM_THREADS="1", MKL_NUM_THREADS="1")
    jobs = [(v, c) for v in variants for c in range(chains)]
    out = {}
    running = []
    os.makedirs("/tmp/gst_theta_bias", exist_ok=True)
    while jobs or running:
        while jobs and len(running) < nproc:
            v, c = jobs.pop(0)
            p = f"/tmp/gst_theta_bias/{dataset}_{v}_{c}.npz"
            running.append((v, c, p, subprocess.Popen(
                [sys.executable, __file__, "--worker", dataset, "beta", v, str(sweeps),
                 str(31000 + c), p], env=env)))
        time.sleep(1.0)
        for item in list(running):
            v, c, p, proc = item
            if proc.poll() is not None:
                assert proc.returncode == 0, (v, c)
                running.remove(item)
                out.setdefault(v, []).append(dict(np.load(p)))
    res = {"dataset": dataset, "sweeps": sweeps, "chains": chains, "burn": BURN,
           "thin": THIN, "variants": {}}
    for v in variants:
        means = np.array([o["theta"].mean() for o in out[v]])
        nus = np.array([o["nu"].mean() for o in out[v]])
        res["variants"][v] = dict(
            theta_mean=float(means.mean()),
            theta_se=float(means.std(ddof=1) / math.sqrt(len(means))),
            theta_chain_means=[float(m) for m in means],
            nu_mean=float(nus.mean()), nu_se=float(nus.std(ddof=1) / math.sqrt(len(nus))),
            secs_per_chain=float(np.mean([o["secs"] for o in out[v]])))
        np.savez_compressed(f"/tmp/gst_theta_bias/{dataset}_{v}_all.npz",
                            theta=np.stack([o["theta"] for o in out[v]]),
                            nu=np.stack([o["nu"] for o in out[v]]),
                            x=np.stack([o["x"] for o in out[v]]))
        print(v, json.dumps(res["variants"][v]), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
