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


def test_general_white_noise_model():
    """Per-backend efac / equad / ECORR (the notebook's J1643-1224 model, with
    enterprise's by_backend selection): parameter names sorted as enterprise sorts them,
    N0 per TOA from its backend's parameters, ECORR columns = observing epochs with >= 2
    TOAs, each with prior variance 10^(2 log10_ecorr) of its backend."""
    psr = data.multiband(nepochs=20, nsub=3)
    pta = model.PTA(psr, components=10, efac=(0.2, 10.0), selection="backend",
                    log10_ecorr=(-8.5, -5.0))
    assert pta.param_names == sorted(pta.param_names) and len(pta.params) == 8
    assert pta.n_ecorr == 20 and pta.nbackend == 2 and pta.m == 20 + pta.ntm + 20
    U = pta.T[:, -20:]
    assert np.all(U.sum(axis=0) == 3) and np.all(U.sum(axis=1) == 1)   # one epoch per TOA
    x = {p.name: v for p, v in zip(pta.params, [1.5, -6.0, -6.5, 0.8, -7.0, -7.5, 4.0, -14.0])}
    n0 = pta.get_ndiag(x)[0]
    bk = pta.bidx
    ef = np.where(bk == 0, 1.5, 0.8)
    eq = np.where(bk == 0, -6.5, -7.5)
    np.testing.assert_array_equal(n0, ef ** 2 * pta._toaerrs ** 2 + 10 ** (2 * eq))
    phi = pta.get_phi(x)[0][-20:]
    np.testing.assert_array_equal(phi, 10 ** (2 * np.where(pta.ecorr_backend == 0, -6.0, -7.0)))
    hind, wind = model.hyper_white_indices(pta.param_names)
    assert [pta.param_names[i] for i in hind] == ["MB_ASP_log10_ecorr", "MB_GUPPI_log10_ecorr",
                                                  "MB_gamma", "MB_log10_A"]
    assert len(wind) == 4
    # quantization: TOAs within 1 s share an epoch, epochs with one TOA get no column
    q = model.quantization_matrix(np.array([0.0, 0.5, 10.0, 20.0, 20.2]))
    np.testing.assert_array_equal(q, [[1, 0], [1, 0], [0, 0], [0, 1], [0, 1]])
