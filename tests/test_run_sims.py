"""run_sims.py grid construction (CPU): entries, ragged twins, initial states, layout."""
import os

import numpy as np

from gibbs_student_t_amd import run_sims


def test_grid_matches_run_sims_structure():
    e = run_sims.build_grid(thetas=(0.05, 0.1), realisations=1)
    # per theta: outlier + no_outlier pulsars, 5 models each (run_sims.py:36,80,86-107)
    assert len(e) == 2 * 2 * 5
    assert [x.model for x in e[:5]] == list(run_sims.MODELS)
    out = [x for x in e if x.kind == "outlier"]
    clean = [x for x in e if x.kind == "no_outlier"]
    assert all(x.pta.n == 130 for x in out)
    for o, c in zip(out, clean):
        assert o.idx == c.idx and o.theta == c.theta
        # simulate_data.py:35-37 deletes the outlier TOAs from the twin
        assert c.pta.n == 130 - int(o.meta["z_true"].sum())
        assert c.pta.T.shape[1] == o.pta.T.shape[1] == 74
    assert e[0].outdir("/x") == os.path.join("/x", "output_outlier", "vvh17", "0.05",
                                             str(e[0].idx))


def test_grid_is_deterministic_and_dof_variant():
    a = run_sims.build_grid(thetas=(0.1,), realisations=2, models=("beta",), dofs=(None, 4.0))
    b = run_sims.build_grid(thetas=(0.1,), realisations=2, models=("beta",), dofs=(None, 4.0))
    assert len(a) == 2 * 2 * 2
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x.pta.get_residuals()[0], y.pta.get_residuals()[0])
    assert a[2].dof == 4.0 and "t4" in a[2].outdir("/r")


def test_initial_state_per_model():
    e = run_sims.build_grid(thetas=(0.05,), realisations=1)
    nst = max(x.pta.n for x in e)
    for x in e:
        s = run_sims.initial_state(x, 3, 0, 1, nst)
        n = x.pta.n
        z0 = 1.0 if x.cfg["model"] in ("t", "mixture", "vvh17") else 0.0   # gibbs.py:50-51
        assert np.all(s["z"][:, :n] == z0) and np.all(s["z"][:, n:] == 0)
        a0 = 1e10 if x.model == "vvh17" else 1.0                           # gibbs.py:44-47
        assert np.all(s["alpha"][:, :n] == a0)
        lo = np.array([p.pmin for p in x.pta.params])
        hi = np.array([p.pmax for p in x.pta.params])
        assert np.all((s["x"] >= lo) & (s["x"] <= hi))
        assert s["theta"][0] == 0.01 and s["nu"][0] == 4.0
