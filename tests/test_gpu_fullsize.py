"""BASELINE.json configs[4] at full size: 100k TOAs, m = 420 (300 timing/DMX + 120 Fourier
columns), run_sims 'beta' mixture model, on the large-model kernel path.

The reference fixtures stop at n = 1500, m = 180 (the oracle must finish in seconds); at the
full size the checks are the likelihood methods (gibbs.py:262-284 and 288-329, i.e. the
per-chain Gram over all 100k TOAs, the timing-model elimination and the Fourier-block
factorization of the large path) against the oracle at states the GPU sampler itself
reached, <= 1e-10 relative, plus the sampler's own invariants (status, finiteness, the
start-of-sweep record).  Parity of these kernels with the reference at the fixture sizes is
in test_gpu_parity.py; this file pins that nothing changes with size.
"""
import warnings

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a HIP device", allow_module_level=True)

from gibbs_student_t_amd._abi import STATUS_ERRORS, STATUS_FLOOR  # noqa: E402
from gibbs_student_t_amd import Gibbs, data  # noqa: E402
from gibbs_student_t_amd.model import PTA  # noqa: E402
from oracle.gibbs_oracle import ChainState, Oracle, OutlierModel  # noqa: E402

KW = dict(model="mixture", vary_df=True, theta_prior="beta")   # run_sims.py:98-99


@pytest.fixture(scope="module")
def big():
    psr = data.scaled_synthetic(n=100_000, components=60, ntm=300, seed=5)
    return PTA(psr, components=60)


def test_fullsize_sampler_and_likelihoods(big):
    pta = big
    n, m = pta.T.shape
    assert (n, m) == (100_000, 420)
    g = Gibbs(pta, **KW, nchains=2, seed=17)
    assert g._native.path == "large"
    rng = np.random.default_rng(3)
    lo = np.array([p.pmin for p in pta.params])
    hi = np.array([p.pmax for p in pta.params])
    x0 = np.stack([rng.uniform(lo, hi) for _ in range(2)])
    x = g.sample(x0, niter=4)
    assert np.all((g.status & STATUS_ERRORS) == 0)
    assert g.chain.shape == (2, 4, len(pta.params)) and g.zchain.shape == (2, 4, n)
    np.testing.assert_array_equal(g.chain[:, 0], x0)          # start-of-sweep record
    assert np.all(np.isfinite(g.bchain)) and np.all(np.isfinite(g.alphachain))
    # some TOAs flagged as outliers, not all (5% injected)
    zf = g._z_all.mean(axis=1)
    assert np.all((zf > 0.0) & (zf < 0.5)), zf

    orc = Oracle(pta, OutlierModel(**KW))
    xe = np.stack([x, np.stack([rng.uniform(lo, hi) for _ in range(2)])])   # (2 points, C, P)
    for xq in xe:
        w, h = g.get_lnlikelihood_white(xq), g.get_lnlikelihood(xq)
        for c in range(2):
            st = ChainState(b=g._b_all[c].copy(), z=g._z_all[c].copy(),
                            alpha=g._alpha_all[c].copy(), pout=g._pout_all[c].copy(),
                            theta=float(g._theta_all[c]), nu=float(g._tdf_all[c]))
            with warnings.catch_warnings():
                warnings.simplefilter("ignore")
                w_ref = orc.lnlike_white(st, xq[c])
                orc.cache = None
                h_ref = orc.lnlike_marginal(st, xq[c])
            assert abs(w[c] - w_ref) <= 1e-10 * abs(w_ref), (c, w[c], w_ref)
            if np.isfinite(h_ref):
                assert abs(h[c] - h_ref) <= 1e-10 * abs(h_ref), (c, h[c], h_ref)
            else:
                assert h[c] == h_ref
    g.close()
