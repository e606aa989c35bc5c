"""CPU ORACLE -- test infrastructure only, never shipped, never measured as the product.

Only ``tests/`` may import this module.  NumPy restatement of the batched synthetic-pulsar
generator (``gibbs_student_t_amd/csrc/gst_sim.hpp``), which restates the reference's
``simulate_data.py:10-39`` recipe:

    err  = 10^(-7 + 0.2 xi)                          simulate_data.py:15
    red  = F (sqrt(phi) xi_red)                      simulate_data.py:21 (ts.add_rednoise,
                                                     A = 1e-14, gamma = 4.33, 30 components)
    z    ~ Bernoulli(theta)                          simulate_data.py:24
    r    = red + ((1 - z) err + z sigma_out) xi      simulate_data.py:26
    r   -= U (U^T r)                                 the refit of the re-read tim file
    clean: outlier TOAs deleted, refit on the rest   simulate_data.py:35-37

with the same Philox4x32-10 stream as the kernel (counter (index, tag, 0xFFFFFFFF, dataset),
key = seed; ``philox`` is checked against the Random123 known-answer vectors in
tests/test_sim_oracle.py).  The reference generator itself needs libstempo/tempo2 (absent
offline): its variates cannot be reproduced, so parity with the reference's *draws* is
unpinned; what is pinned is the recipe (the formulas above, line by line) and the kernel's
agreement with this restatement.
"""
from __future__ import annotations

import math

import numpy as np

M32 = np.uint64(0xFFFFFFFF)
TAG_SIM_RED, TAG_SIM_ERR, TAG_SIM_Z, TAG_SIM_XI, TAG_SIM_T = (k << 24 for k in (8, 9, 10, 11, 12))
SIM_SWEEP = 0xFFFFFFFF


def philox(c0, c1, c2, c3, k0, k1):
    """Philox4x32-10 on arrays of 32-bit counters (numpy uint64 carriers)."""
    c = [np.asarray(x, dtype=np.uint64) & M32 for x in (c0, c1, c2, c3)]
    c = list(np.broadcast_arrays(*c))
    c = [x.copy() for x in c]
    k0 = np.uint64(k0) & M32
    k1 = np.uint64(k1) & M32
    M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
    W0, W1 = np.uint64(0x9E3779B9), np.uint64(0xBB67AE85)
    for _ in range(10):
        p0 = M0 * c[0]
        p1 = M1 * c[2]
        n0 = (p1 >> np.uint64(32)) ^ c[1] ^ k0
        n2 = (p0 >> np.uint64(32)) ^ c[3] ^ k1
        c = [n0, p1 & M32, n2, p0 & M32]
        k0 = (k0 + W0) & M32
        k1 = (k1 + W1) & M32
    return c


def u01(lo, hi):
    x = (np.asarray(hi, dtype=np.uint64) << np.uint64(32)) | np.asarray(lo, dtype=np.uint64)
    return (x >> np.uint64(11)).astype(np.float64) * 2.0 ** -53


class Stream:
    """Rng of philox.hpp for one dataset: draw(index, tag) -> two uniforms in [0, 1)."""

    def __init__(self, seed, dataset):
        self.k0 = int(seed) & 0xFFFFFFFF
        self.k1 = (int(seed) >> 32) & 0xFFFFFFFF
        self.chain = int(dataset) & 0xFFFFFFFF

    def uniform2(self, index, tag):
        r = philox(index, tag, SIM_SWEEP, self.chain, self.k0, self.k1)
        return u01(r[0], r[1]), u01(r[2], r[3])

    def normal(self, index, tag):
        """Box-Muller, cosine half (gst_kernel.hpp normal_from)."""
        a, b = self.uniform2(index, tag)
        return np.sqrt(-2.0 * np.log(1.0 - a)) * np.cos(2.0 * np.pi * b)

    def gamma(self, a, index, tag):
        """Marsaglia-Tsang Gamma(a, 1) with paired attempts (gst_kernel.hpp gamma_mt)."""
        boost = 1.0
        if a < 1.0:
            ub, _ = self.uniform2(index, tag | 0xFFFFFF)
            boost = math.exp(math.log(1.0 - float(ub)) / a)
            a += 1.0
        d = a - 1.0 / 3.0
        cc = 1.0 / math.sqrt(9.0 * d)
        for att in range(128):
            u1, u2 = (float(x) for x in self.uniform2(index, tag | (2 * att)))
            ua, ub = (float(x) for x in self.uniform2(index, tag | (2 * att + 1)))
            r = math.sqrt(-2.0 * math.log(1.0 - u1))
            for h in range(2):
                xn = r * (math.cos(2 * math.pi * u2) if h == 0 else math.sin(2 * math.pi * u2))
                u3 = ua if h == 0 else ub
                v = 1.0 + cc * xn
                if v <= 0.0:
                    continue
                v = v * v * v
                x2 = xn * xn
                if u3 < 1.0 - 0.0331 * x2 * x2:
                    return d * v * boost
                if math.log(u3) < 0.5 * x2 + d * (1.0 - v + math.log(v)):
                    return d * v * boost
        return d * boost


def simulate(toas_F, U, *, seed, dataset, theta, sigma_out, log10_A=-14.0, gamma=4.33,
             dof=0.0, lf=None, ldf=None, log_fyr=None, red=None, toaerrs=None, clean=True):
    """One dataset: returns (residuals, toaerrs, z, residuals_clean or None).

    ``toas_F`` is the Fourier basis F [n, nf] (ignored when ``red`` is given)."""
    st = Stream(seed, dataset)
    n = U.shape[0]
    t = np.arange(n, dtype=np.uint64)
    if red is None:
        F = toas_F
        nf = F.shape[1]
        lc = 2.0 * log10_A * 2.302585092994045684 - (math.log(12.0) + 2.0 * math.log(math.pi)) \
            + (gamma - 3.0) * log_fyr
        coef = np.sqrt(np.exp(lc - gamma * lf + ldf)) * st.normal(np.arange(nf, dtype=np.uint64),
                                                                  TAG_SIM_RED)
        rt = F @ coef
    else:
        rt = np.asarray(red, dtype=np.float64)
    err = np.asarray(toaerrs, dtype=np.float64) if toaerrs is not None else \
        10.0 ** (-7.0 + st.normal(t, TAG_SIM_ERR) * 0.2)
    uz, _ = st.uniform2(t, TAG_SIM_Z)
    z = (uz < theta).astype(np.float64)
    xi = st.normal(t, TAG_SIM_XI)
    if dof > 0:
        g = np.array([st.gamma(0.5 * dof, i, TAG_SIM_T) for i in range(n)])
        xi = math.sqrt(0.5 * dof) * xi / np.sqrt(g)
    r = rt + ((1.0 - z) * err + z * sigma_out) * xi
    r = r - U @ (U.T @ r)
    r2 = None
    if clean:
        k = z == 0
        Uk = U[k]
        beta = np.linalg.solve(Uk.T @ Uk, Uk.T @ r[k])
        r2 = np.where(k, r - U @ beta, 0.0)
    return r, err, z, r2
