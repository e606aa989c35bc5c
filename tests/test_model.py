"""The structured model against the formulas it restates (enterprise stand-in)."""
import numpy as np
import scipy.special

from gibbs_student_t_amd import data, model


def test_params_sorted_and_roles():
    pta = model.PTA(data.j1713())
    names = pta.param_names
    assert names == sorted(names)
    assert [n.split("_", 1)[1] for n in names] == ["gamma", "log10_A", "log10_equad"]
    hind, wind = model.hyper_white_indices(names)
    assert hind.tolist() == [0, 1] and wind.tolist() == [2]
    pta2 = model.PTA(data.j1713(), efac=(0.2, 10.0))
    hind, wind = model.hyper_white_indices(pta2.param_names)
    assert hind.tolist() == [1, 2] and wind.tolist() == [0, 3]


def test_basis_and_noise():
    psr = data.j1713()
    pta = model.PTA(psr)
    assert pta.T.shape == (130, 74)
    U = pta.T[:, 60:]
    np.testing.assert_allclose(U.T @ U, np.eye(14), atol=1e-10)
    x = dict(zip(pta.param_names, [4.33, -14.0, -7.0]))
    N0 = pta.get_ndiag(x)[0]
    np.testing.assert_allclose(N0, psr.toaerrs ** 2 + 1e-14, rtol=1e-14)
    phiinv, ld = pta.get_phiinv(x, logdet=True)[0]
    phi = pta.get_phi(x)[0]
    np.testing.assert_allclose(phiinv, 1 / phi)
    assert np.isclose(ld, np.sum(np.log(phi)))
    f = pta.Ffreqs[::2]
    want = (1e-14) ** 2 / 12 / np.pi ** 2 * model.FYR ** (4.33 - 3) * f ** -4.33 * f[0]
    np.testing.assert_allclose(phi[:60:2], want, rtol=1e-12)
    assert np.all(phi[60:] == 1e40)


def test_prior_bounds_inclusive():
    p = model.Uniform("x", -10, -5)
    assert p.get_logpdf(-10.0) == p.get_logpdf(-5.0) == -np.log(5.0)
    assert p.get_logpdf(-4.999) == -np.inf


def test_df_tables():
    A, B = model.df_tables(130)
    nu = np.arange(1, 31)
    np.testing.assert_allclose(A, 130 * (nu / 2) * np.log(nu / 2))
    np.testing.assert_allclose(B, 130 * scipy.special.gammaln(nu / 2))


def test_simulate_data_pair():
    out, clean = data.simulate_data(seed=3, theta=0.1)
    z = out.meta["z_true"]
    assert out.n == 130 and clean.n == 130 - z.sum()
    pta = model.PTA(clean)
    assert pta.T.shape[0] == clean.n
