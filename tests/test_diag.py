"""Diagnostics used for the ESS/s metric against closed forms."""
import numpy as np

from gibbs_student_t_amd import diag


def ar1(m, n, rho, rng):
    x = np.zeros((m, n))
    x[:, 0] = rng.standard_normal(m) / np.sqrt(1 - rho ** 2)
    e = rng.standard_normal((m, n))
    for t in range(1, n):
        x[:, t] = rho * x[:, t - 1] + e[:, t]
    return x


def test_bulk_ess_matches_ar1_closed_form():
    rng = np.random.default_rng(1)
    for rho in (0.0, 0.5, 0.9):
        x = ar1(32, 4000, rho, rng)
        want = diag.ar1_ess(rho, 32, 4000)
        got = diag.bulk_ess(x)
        assert abs(got / want - 1) < 0.12, (rho, got, want)


def test_rhat_detects_disagreeing_chains():
    rng = np.random.default_rng(2)
    iid = rng.standard_normal((8, 1000))
    assert diag.split_rhat(iid) < 1.01
    bad = iid + np.arange(8)[:, None] * 0.5
    assert diag.split_rhat(bad) > 1.1


def test_constant_chain_is_nan():
    assert np.isnan(diag.bulk_ess(np.ones((4, 100))))


def test_ess_rhat_equals_separate_functions():
    rng = np.random.default_rng(3)
    x = rng.standard_normal((6, 200)).cumsum(axis=1) * 0.1 + rng.standard_normal((6, 200))
    e, r = diag.ess_rhat(x)
    assert e == diag.bulk_ess(x) and r == diag.split_rhat(x)
