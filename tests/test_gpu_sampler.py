"""The drop-in ``Gibbs`` class (reference gibbs.py:8-385) on the GPU.

Same constructor, methods and chain attributes as the reference; every call runs through
libgst.so.  Likelihood methods are checked against the oracle (<= 1e-10 relative) at the
reference's recorded states; ``sample`` against the reference's chain layout
(gibbs.py:344-361: state at the START of each sweep recorded, shapes per attribute).
"""
import warnings

import numpy as np
import pytest

from golden_io import load_ref, sweep_state

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a HIP device", allow_module_level=True)

from gibbs_student_t_amd._abi import STATUS_ERRORS, STATUS_FLOOR  # noqa: E402
from gibbs_student_t_amd import Gibbs  # noqa: E402
from oracle.gibbs_oracle import ChainState, Oracle, OutlierModel  # noqa: E402


def _load_state(g, s):
    g._b_all[0] = s["b"]
    g._z_all[0] = s["z"]
    g._alpha_all[0] = s["alpha"]
    g._pout_all[0] = s["pout"]
    g._theta_all[0] = s["theta"]
    g._tdf_all[0] = s["nu"]


@pytest.mark.parametrize("name", ["beta_fixed", "t_fixed", "scaled_beta_fixed"])
def test_likelihood_methods_match_oracle(name):
    ref = load_ref(name)
    g = Gibbs(ref["pta"], **ref["kw"], seed=1)
    orc = Oracle(ref["pta"], OutlierModel(**ref["kw"]))
    for i in (0, 3):
        s = sweep_state(ref, i)
        _load_state(g, s)
        st = ChainState(b=s["b"], z=s["z"], alpha=s["alpha"], pout=s["pout"],
                        theta=s["theta"], nu=s["nu"])
        x = ref["chain"][i]
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            w_ref = orc.lnlike_white(st, x)
            orc.cache = None
            h_ref = orc.lnlike_marginal(st, x)
        assert abs(g.get_lnlikelihood_white(x) - w_ref) <= 1e-10 * abs(w_ref)
        assert abs(g.get_lnlikelihood(x) - h_ref) <= 1e-10 * abs(h_ref)
        assert g.get_lnprior(x) == pytest.approx(sum(p.get_logpdf(v) for p, v in
                                                     zip(ref["pta"].params, x)))
    g.close()


@pytest.mark.parametrize("name", ["beta_fixed", "scaled_t_fixed"])
def test_sample_has_reference_layout(name):
    ref = load_ref(name)
    pta = ref["pta"]
    n, m = pta.T.shape
    g = Gibbs(pta, **ref["kw"], seed=7)
    niter = 40
    x = g.sample(ref["xs"], niter=niter)
    assert g.chain.shape == (niter, len(pta.params))
    assert g.bchain.shape == (niter, m)
    for a in (g.zchain, g.alphachain, g.poutchain):
        assert a.shape == (niter, n)
    assert g.thetachain.shape == (niter,) and g.dfchain.shape == (niter,)
    np.testing.assert_array_equal(g.chain[0], ref["xs"])     # start-of-sweep record
    assert np.all(g.bchain[0] == 0.0)                         # gibbs.py:36 initial b
    z0 = 1.0 if ref["kw"]["model"] in ("t", "mixture", "vvh17") else 0.0
    assert np.all(g.zchain[0] == z0)                          # gibbs.py:50-51
    assert np.all(np.isfinite(g.chain)) and np.all(np.isfinite(g.bchain))
    assert x.shape == (len(pta.params),) and np.all((g.status & STATUS_ERRORS) == 0)
    assert set(np.unique(g.zchain)) <= {0.0, 1.0}
    assert np.all((g.dfchain >= 1) & (g.dfchain <= 30))
    g.close()


def test_stage_methods_and_reproducibility():
    ref = load_ref("uniform_fixed")
    runs = []
    for seed in (11, 11, 12):
        g = Gibbs(ref["pta"], **ref["kw"], seed=seed)
        x = ref["xs"]
        # one sweep written out as the reference's loop body (gibbs.py:367-380)
        x = g.update_white_params(x)
        x = g.update_hyper_params(x)
        g._b = b = g.update_b(x)
        g._theta = th = g.update_theta(x)
        g._z = z = g.update_z(x)
        g._alpha = a = g.update_alpha(x)
        g.tdf = nu = g.update_df(x)
        assert b.shape == (ref["pta"].T.shape[1],) and z.shape == a.shape == (ref["pta"].n,)
        assert 0.0 <= th <= 1.0 and 1 <= nu <= 30
        runs.append((x.copy(), b.copy(), z.copy(), a.copy()))
        g.close()
    for u, v in zip(runs[0], runs[1]):
        np.testing.assert_array_equal(u, v)                   # same seed: same chain
    assert not np.array_equal(runs[0][1], runs[2][1])         # other seed: other draw


def test_stage_methods_return_without_committing():
    """gibbs.py:145-259: update_b/theta/z/alpha/df RETURN draws; the latent state changes
    only when the caller assigns it (gibbs.py:374-380); update_z records _pout (:225)."""
    ref = load_ref("beta_fixed")
    g = Gibbs(ref["pta"], **ref["kw"], seed=5)
    s = sweep_state(ref, 3)
    _load_state(g, s)
    x = ref["chain"][3]
    before = {k: np.array(getattr(g, k), copy=True) for k in ("_b", "_z", "_alpha", "_theta",
                                                               "tdf", "_pout")}
    b1, b2 = g.update_b(x), g.update_b(x)
    th1, th2 = g.update_theta(x), g.update_theta(x)
    a1 = g.update_alpha(x)
    nu1 = g.update_df(x)
    for k in ("_b", "_z", "_alpha", "_theta", "tdf", "_pout"):
        np.testing.assert_array_equal(getattr(g, k), before[k], err_msg=k)
    assert not np.array_equal(b1, b2) and th1 != th2          # fresh draws per call
    assert a1.shape == s["alpha"].shape and 1 <= nu1 <= 30
    orc = Oracle(ref["pta"], OutlierModel(**ref["kw"]))

    def pout_oracle():
        st = ChainState(b=np.array(g._b), z=np.array(g._z), alpha=np.array(g._alpha),
                        pout=np.array(g._pout), theta=float(g._theta), nu=float(g.tdf))
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            return orc.outlier_prob(st, x)

    z1 = g.update_z(x)
    np.testing.assert_array_equal(g._z, before["_z"])          # z not committed ...
    np.testing.assert_allclose(g._pout, pout_oracle(), rtol=1e-10, atol=0)   # ... _pout is
    assert set(np.unique(z1)) <= {0.0, 1.0}
    # the reference's sweep commits by assignment; later stages then see the new values
    g._b = b1
    g._theta = th1
    np.testing.assert_array_equal(g._b, b1)
    g.update_z(x)
    np.testing.assert_allclose(g._pout, pout_oracle(), rtol=1e-10, atol=0)
    # get_lnlikelihood_df (gibbs.py:331-335) per chain
    assert np.isclose(g.get_lnlikelihood_df(4), orc.df_logdensity(
        ChainState(b=g._b, z=g._z, alpha=g._alpha, pout=g._pout, theta=g._theta, nu=4), 4),
        rtol=1e-12)
    g.close()


def test_batched_chains_and_thinning():
    ref = load_ref("beta_fixed")
    C, niter, every = 8, 30, 4
    g = Gibbs(ref["pta"], **ref["kw"], nchains=C, seed=3, record_every=every, chunk=8)
    x = g.sample(ref["xs"], niter=niter)
    nrec = (niter + every - 1) // every
    assert x.shape == (C, 3)
    assert g.chain.shape == (C, nrec, 3) and g.zchain.shape == (C, nrec, ref["pta"].n)
    np.testing.assert_array_equal(g.chain[:, 0], np.tile(ref["xs"], (C, 1)))
    assert np.std(g.chain[:, -1, 0]) > 0                      # chains are independent
    g.close()


@pytest.mark.parametrize("name", ["beta_fixed", "vvh17_fixed"])
def test_checkpoint_resume_is_bitwise(name, tmp_path):
    """sample(N) -> save_checkpoint -> a NEW sampler -> load_checkpoint -> sample(M) gives
    the chains of one sample(N + M) run, bitwise (chain arrays, final state)."""
    ref = load_ref(name)
    N, M, C = 30, 20, 4
    g = Gibbs(ref["pta"], **ref["kw"], nchains=C, seed=4242, chunk=16)
    xa = g.sample(ref["xs"], niter=N + M)
    full = {k: getattr(g, k).copy() for k in ("chain", "bchain", "zchain", "alphachain",
                                               "poutchain", "thetachain", "dfchain")}
    g.close()
    h = Gibbs(ref["pta"], **ref["kw"], nchains=C, seed=4242, chunk=16)
    h.sample(ref["xs"], niter=N)
    h.save_checkpoint(tmp_path / "ck.npz")
    h.close()
    r = Gibbs(ref["pta"], **ref["kw"], nchains=C, seed=1)     # key comes from the file
    x = r.load_checkpoint(tmp_path / "ck.npz")
    xb = r.sample(x, niter=M)
    for k, v in full.items():
        np.testing.assert_array_equal(getattr(r, k), v[:, N:], err_msg=k)
    np.testing.assert_array_equal(xb, xa)
    r.close()


def test_checkpoint_refuses_stale_pairs_and_other_datasets(tmp_path):
    """A stage call after sample() advances the Philox counter past the sampled x: the
    checkpoint would not resume the uninterrupted chain, so it is refused.  A
    checkpoint loads only on the dataset it was taken on."""
    ref = load_ref("beta_fixed")
    g = Gibbs(ref["pta"], **ref["kw"], nchains=2, seed=7)
    x = g.sample(ref["xs"], niter=5)
    g.save_checkpoint(tmp_path / "ok.npz")
    g.update_theta(x)
    with pytest.raises(RuntimeError, match="directly follow"):
        g.checkpoint()
    g.close()
    other = load_ref("c3_beta_fixed")
    h = Gibbs(other["pta"], **ref["kw"], nchains=2, seed=7)
    if other["pta"].get_basis()[0].shape == ref["pta"].get_basis()[0].shape:
        with pytest.raises(ValueError, match="different dataset"):
            h.load_checkpoint(tmp_path / "ok.npz")
    else:
        with pytest.raises(ValueError):
            h.load_checkpoint(tmp_path / "ok.npz")
    h.close()
