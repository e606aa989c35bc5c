"""Pin the CPU oracle against golden vectors produced by running the reference itself.

Fixtures: tests/golden/ref_*.npz (tools/gen_golden.py; reference gibbs.py:8-385 run with
the build's model, seeded, with every variate recorded).
"""
import warnings

import numpy as np
import pytest

from golden_io import CHAIN_KEYS, fixture_names, load_ref, sweep_state, sweep_tape
from oracle.gibbs_oracle import (ChainState, LegacyNumpyVariates, Oracle, OutlierModel,
                                 TapeVariates, bernoulli_from_uniform, choice_from_uniform,
                                 initial_state)

NAMES = fixture_names()


def _oracle(ref):
    return Oracle(ref["pta"], OutlierModel(**ref["kw"]))


@pytest.mark.parametrize("name", NAMES)
def test_legacy_stream_reproduces_reference_bit_exact(name):
    """Same seed, same RNG calls in the same order -> identical chains (gibbs.py:342-385)."""
    ref = load_ref(name)
    orc = _oracle(ref)
    np.random.seed(int(ref["seed"]))
    if int(ref["prior_draw"]):
        xs = ref["pta"].sample_params()
    else:
        xs = ref["xs"]
    np.testing.assert_array_equal(xs, ref["xs"])
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        out, st, x = orc.run(xs, int(ref["niter"]))
    for k in CHAIN_KEYS:
        np.testing.assert_array_equal(out[k], ref[k], err_msg=k)
    np.testing.assert_array_equal(st.b, ref["final_b"])
    np.testing.assert_array_equal(st.alpha, ref["final_alpha"])


@pytest.mark.parametrize("name", NAMES)
def test_tape_replay_per_sweep(name):
    """Each sweep re-run from the recorded start state with the recorded variates."""
    ref = load_ref(name)
    orc = _oracle(ref)
    niter = int(ref["niter"])
    for i in range(niter):
        s0, s1 = sweep_state(ref, i), sweep_state(ref, i + 1)
        st = ChainState(b=s0["b"].copy(), z=s0["z"].copy(), alpha=s0["alpha"].copy(),
                        pout=s0["pout"].copy(), theta=s0["theta"], nu=s0["nu"])
        trace = {}
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            x1 = orc.sweep(st, s0["x"], TapeVariates(sweep_tape(ref, i)), trace=trace)
        tape = sweep_tape(ref, i)
        np.testing.assert_array_equal(trace["x_white"], tape["x_white"])
        if i + 1 < niter:
            np.testing.assert_array_equal(x1, ref["chain"][i + 1])
        np.testing.assert_array_equal(st.b, s1["b"])
        np.testing.assert_array_equal(np.asarray(st.z, float), s1["z"])
        np.testing.assert_array_equal(st.alpha, s1["alpha"])
        np.testing.assert_array_equal(st.pout, s1["pout"])
        assert st.theta == s1["theta"] and float(st.nu) == s1["nu"]
        wl = np.array([v for _, v in trace["white_log"]])
        hl = np.array([v for _, v in trace["hyper_log"]])
        np.testing.assert_array_equal(wl, tape["white_lnl"])
        np.testing.assert_array_equal(hl, tape["hyper_lnl"])


def test_initial_state_matches_reference_layout():
    ref = load_ref("beta_fixed")
    st = initial_state(ref["pta"], OutlierModel(**ref["kw"]))
    s0 = sweep_state(ref, 0)
    np.testing.assert_array_equal(st.z, s0["z"])
    np.testing.assert_array_equal(st.alpha, s0["alpha"])
    assert st.theta == s0["theta"] and st.nu == s0["nu"]


def test_choice_mapping_matches_numpy():
    rs = np.random.RandomState(7)
    p = np.array([0.1, 0.15, 0.5, 0.15, 0.1])
    a = [0.1, 0.5, 1.0, 3.0, 10.0]
    for _ in range(2000):
        st = rs.get_state()
        v = rs.choice(a, p=p)
        rs.set_state(st)
        u = rs.random_sample()
        assert choice_from_uniform(a, p, u) == v


def test_bernoulli_mapping_matches_numpy():
    rs = np.random.RandomState(11)
    q = np.concatenate([rs.random_sample(3000), [0.0, 1.0, 0.5, 1e-300, 1 - 1e-16]])
    st = rs.get_state()
    z = rs.binomial(1, q)
    rs.set_state(st)
    for qi, zi in zip(q, z):
        u = rs.random_sample() if qi != 0.0 else np.nan
        assert bernoulli_from_uniform(qi, u) == zi
