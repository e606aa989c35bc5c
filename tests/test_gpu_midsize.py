"""Mid-size pulsars on the large path: the one-wave-per-chain kernels against the
generic ones they replace, at n = 1000 (the large path forced: since round 3 the persistent
kernel's 16-slot instance takes pulsars of up to 1024 TOAs).

* lg_gram_small must give bitwise lg_gram's Gram: whole chains are compared bitwise with the
  generic Gram forced (GST_DEBUG_LARGE_GRAM).
* lg_hyper_reg runs the same MH with another elimination: likelihoods within rounding, the
  same discrete draws, continuous draws within 1e-8 (GST_DEBUG_LARGE_HYPER).

The kernels' parity with the reference itself is covered by the large-path replays of
test_gpu_parity.py, whose fixtures (m = 74) run on these same kernels.
"""
import numpy as np
import pytest

from gibbs_student_t_amd._abi import STATUS_ERRORS, STATUS_FLOOR  # noqa: E402
from gibbs_student_t_amd import data
from gibbs_student_t_amd.model import PTA
from gibbs_student_t_amd.native import NativeSampler

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

CFG = dict(model="mixture", vary_df=True, theta_prior="beta")
C, S = 16, 6


@pytest.fixture(scope="module")
def pta():
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    return PTA(data.scaled_synthetic(n=1000, components=30, ntm=14, seed=11), components=30)


def _run(pta, **debug):
    ns = NativeSampler(pta, CFG, 0, path="large")   # n <= 1024 would pick the persistent kernel
    ns.set_debug(**debug)
    ns.alloc(C)
    rng = np.random.default_rng(5)
    lo = np.array([p.pmin for p in pta.params])
    hi = np.array([p.pmax for p in pta.params])
    x0 = rng.uniform(lo, hi, size=(C, len(lo)))
    ns.set_state(x=x0, z=np.zeros((C, ns.n)), alpha=np.ones((C, ns.n)),
                 theta=np.full(C, 0.05), nu=np.full(C, 4.0))
    lnl = ns.eval_lnlike()
    rec = ns.alloc_records(S)
    ns.sweep(S, records=rec, seed=21)
    out = {k: v.cpu().numpy() for k, v in rec.items()}
    out["status"] = ns.get_state()["status"]
    ns.close()
    return lnl, out


def test_small_gram_is_bitwise_the_supertile_gram(pta):
    lnl_a, a = _run(pta)
    lnl_b, b = _run(pta, large_gram=True)
    assert np.all((a["status"] & STATUS_ERRORS) == 0) and np.all((b["status"] & STATUS_ERRORS) == 0)
    for k in a:
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
    for u, v in zip(lnl_a, lnl_b):
        np.testing.assert_array_equal(np.asarray(u), np.asarray(v))


def test_register_hyper_matches_lds_hyper(pta):
    lnl_a, a = _run(pta)
    lnl_b, b = _run(pta, large_hyper=True)
    assert np.all((a["status"] & STATUS_ERRORS) == 0) and np.all((b["status"] & STATUS_ERRORS) == 0)
    # white lnL: same kernel; hyper (b-marginalised) lnL: two eliminations of one matrix
    np.testing.assert_array_equal(np.asarray(lnl_a[0]), np.asarray(lnl_b[0]))
    h_a, h_b = np.asarray(lnl_a[1]), np.asarray(lnl_b[1])
    assert np.all(np.abs(h_a - h_b) <= 1e-11 * np.abs(h_b)), np.max(np.abs(h_a - h_b) / np.abs(h_b))
    for k in ("x", "z", "nu"):
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
    # b normwise per chain-sweep (its small components carry cond(Sigma) x eps of the two
    # eliminations' rounding: the scaled fixture's 120-column block reaches cond ~ 1e10)
    eb = np.linalg.norm(a["b"] - b["b"], axis=-1) / np.maximum(np.linalg.norm(b["b"], axis=-1),
                                                                1e-300)
    assert np.all(eb <= 1e-8), ("b", eb.max())
    for k in ("alpha", "pout", "theta"):
        d = np.abs(a[k] - b[k])
        assert np.all(d <= 1e-8 * np.maximum(np.abs(b[k]), 1e-300) + 1e-300), (k, d.max())


@pytest.mark.parametrize("name", ["ecb_beta_fixed", "ecb_uniform_fixed", "ecn_t_fixed",
                                  "ecn_vvh17_fixed", "scaled_beta_fixed"])
def test_register_hyper_matches_lds_hyper_ecorr(name):
    """lg_hyper_reg's ECORR and per-backend branches (phi^-1 of the ECORR columns from their
    backend's log10_ecorr, the ECORR log|phi| term, the b draw over ECORR columns) against
    lg_hyper on reference fixtures with 44 hyper columns (20 Fourier + 24 ECORR epochs:
    lg_hyper_reg<8>) and 120 (scaled: 60 components: lg_hyper_reg<16>, two columns per lane;
    mb's 20 + 60 ECORR columns take lg_hyper<2>, the tests below); their parity with the
    reference itself is test_gpu_parity.py's large-path replays."""
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    from golden_io import load_ref, sweep_state
    ref = load_ref(name)
    s0 = sweep_state(ref, 0)
    outs = []
    for large_hyper in (False, True):
        ns = NativeSampler(ref["pta"], ref["kw"], 0, path="large")
        ns.set_debug(large_hyper=large_hyper)
        ns.alloc(C)
        ns.set_state(x=np.tile(ref["xs"], (C, 1)), b=np.tile(s0["b"], (C, 1)),
                     z=np.tile(s0["z"], (C, 1)), alpha=np.tile(s0["alpha"], (C, 1)),
                     pout=np.tile(s0["pout"], (C, 1)), theta=np.full(C, s0["theta"]),
                     nu=np.full(C, s0["nu"]))
        rec = ns.alloc_records(S)
        ns.sweep(S, records=rec, seed=33)
        out = {k: v.cpu().numpy() for k, v in rec.items()}
        out["status"] = ns.get_state()["status"]
        ns.close()
        outs.append(out)
    a, b = outs
    assert np.all((a["status"] & STATUS_ERRORS) == 0)
    np.testing.assert_array_equal(a["status"], b["status"])
    for k in ("x", "z", "nu"):
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
    # b normwise per chain-sweep (its small components carry cond(Sigma) x eps of the two
    # eliminations' rounding: the scaled fixture's 120-column block reaches cond ~ 1e10)
    eb = np.linalg.norm(a["b"] - b["b"], axis=-1) / np.maximum(np.linalg.norm(b["b"], axis=-1),
                                                                1e-300)
    assert np.all(eb <= 1e-8), ("b", eb.max())
    for k in ("alpha", "pout", "theta"):
        d = np.abs(a[k] - b[k])
        assert np.all(d <= 1e-8 * np.maximum(np.abs(b[k]), 1e-300) + 1e-300), (k, d.max())


@pytest.mark.parametrize("name", ["ebig_beta_fixed", "ebig_t_fixed", "mb_beta_fixed",
                                  "mbn_vvh17_fixed"])
def test_epochs_first_hyper_matches_blocked_hyper(name):
    """ebig (20 Fourier + 130 ECORR epochs, 14 timing-model columns) and mb / mbn (20 + 60):
    the epochs-first elimination lg_hyper<2> (hyper class 2, their default) against the
    generic kernel GST_DEBUG_LARGE_HYPER forces (ebig: the blocked global-memory lg_hyper<1>;
    mb: the LDS-resident lg_hyper<0>) -- the b-marginalised likelihood at 256 states (prior
    draws of x, the fixture's latents) within 1e-10 relative.  The two factor Sigma in
    different orders, so their Philox b draws are different (equally distributed) draws and
    the chains are compared with the reference instead: test_gpu_parity.py's large-path
    likelihood, MH / b-draw (recorded draw term) and replay tests run on lg_hyper<2>."""
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    from golden_io import load_ref, sweep_state
    ref = load_ref(name)
    pta = ref["pta"]
    s0 = sweep_state(ref, 0)
    C2 = 256
    lo = np.array([p.pmin for p in pta.params])
    hi = np.array([p.pmax for p in pta.params])
    x = np.random.default_rng(5).uniform(lo, hi, size=(C2, len(lo)))
    got = []
    for large_hyper in (False, True):
        ns = NativeSampler(pta, ref["kw"], 0, path="large")
        ns.set_debug(large_hyper=large_hyper)
        ns.alloc(C2)
        ns.set_state(x=x, b=np.tile(s0["b"], (C2, 1)), z=np.tile(s0["z"], (C2, 1)),
                     alpha=np.tile(s0["alpha"], (C2, 1)), pout=np.tile(s0["pout"], (C2, 1)),
                     theta=np.full(C2, s0["theta"]), nu=np.full(C2, s0["nu"]))
        w, h = ns.eval_lnlike()
        got.append((np.asarray(w), np.asarray(h)))
        ns.close()
    (w2, h2), (w1, h1) = got
    np.testing.assert_array_equal(w2, w1)
    ok = np.isfinite(h1)
    assert ok.sum() > C2 // 2
    np.testing.assert_array_equal(np.isfinite(h2), ok)
    r = np.abs(h2[ok] - h1[ok]) / np.abs(h1[ok])
    assert r.max() <= 1e-10, r.max()


@pytest.mark.parametrize("dataset", ["ebig", "mb"])
def test_epochs_first_hyper_draws_match_blocked_hyper(dataset):
    """The two eliminations' Philox b draws are different draws of one law, so chains of the
    same start through lg_hyper<2> and the generic kernel must have the same marginal law at
    every sweep (converged or not): 1024 chains from prior draws, after 150 sweeps, every
    sampled parameter plus theta, nu and two b components, two-sample KS p > 1e-3."""
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    import scipy.stats
    from golden_io import load_dataset
    from gibbs_student_t_amd.run_sims import MODELS
    pta = load_dataset(dataset=dataset)
    C2, S2 = 1024, 150
    lo = np.array([p.pmin for p in pta.params])
    hi = np.array([p.pmax for p in pta.params])
    x0 = np.random.default_rng(9).uniform(lo, hi, size=(C2, len(lo)))
    fin = []
    for large_hyper in (False, True):
        ns = NativeSampler(pta, MODELS["beta"], 0, path="large")
        ns.set_debug(large_hyper=large_hyper)
        ns.alloc(C2)
        ns.set_state(x=x0, z=np.zeros((C2, pta.n)), alpha=np.ones((C2, pta.n)),
                     theta=np.full(C2, 0.05), nu=np.full(C2, 4.0))
        ns.sweep(S2, seed=91)
        st = ns.get_state()
        ns.close()
        assert np.all((st["status"] & STATUS_ERRORS) == 0)
        fin.append(st)
    a, b = fin
    series = [(f"x{j}", a["x"][:, j], b["x"][:, j]) for j in range(len(lo))]
    series += [("theta", a["theta"], b["theta"]), ("nu", a["nu"], b["nu"]),
               ("b_fourier0", a["b"][:, 0], b["b"][:, 0]), ("b_last", a["b"][:, -1], b["b"][:, -1])]
    for nm, u, v in series:
        p = scipy.stats.ks_2samp(u, v).pvalue
        assert p > 1e-3, f"{nm}: KS p = {p:.2e} (means {u.mean():.4g} / {v.mean():.4g})"


def test_overlapping_ecorr_epochs_take_the_general_elimination():
    """lg_hyper<2> eliminates ECORR epochs first because disjoint epochs make the ECORR block
    of T^T N^-1 T diagonal.  A basis where TOAs sit in two ECORR columns
    (nothing enforced it) must run the general elimination instead: the ebig
    dataset with every 5th TOA also in the next epoch's column, on the large path, gives the
    b-marginalised likelihood of the oracle (gibbs.py:288-329) at 64 prior draws, within
    1e-9 relative or the fp64 oracle's own error against the long-double evaluation; the
    disjoint original keeps the epochs-first kernel, same check."""
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    import os
    import warnings
    from golden_io import GOLDEN
    from oracle.gibbs_oracle import (ChainState, Oracle, OutlierModel,
                                     lnlike_marginal_extended)
    from gibbs_student_t_amd.run_sims import MODELS
    d = dict(np.load(os.path.join(GOLDEN, "ebig_dataset.npz"), allow_pickle=False))
    nec = int(d["n_ecorr"])
    for overlap in (False, True):
        T = d["T"].copy()
        m = T.shape[1]
        if overlap:
            ec = T[:, m - nec:]
            for t in range(0, T.shape[0], 5):
                e = int(np.flatnonzero(ec[t])[0]) if ec[t].any() else 0
                e2 = (e + 1) % nec
                if ec[:, e2].any():
                    T[t, m - nec + e2] = 1.0
            assert ((T[:, m - nec:] != 0).sum(axis=1) > 1).any()
        name = str(d["names"][0]).split("_")[0]
        pta = PTA.from_arrays(name, d["residuals"], d["toaerrs"], T, d["Ffreqs"],
                              int(d["components"]), float(d["tm_weight"]),
                              efac=(0.2, 10.0) if int(d["efac_varied"]) else 1.0,
                              backends=d["backends"], selection=str(d["selection"]),
                              n_ecorr=nec, ecorr_backend=d["ecorr_backend"],
                              log10_ecorr=tuple(d["log10_ecorr"]) or None)
        C2 = 64
        lo = np.array([p.pmin for p in pta.params])
        hi = np.array([p.pmax for p in pta.params])
        x = np.random.default_rng(8).uniform(lo, hi, size=(C2, len(lo)))
        ns = NativeSampler(pta, MODELS["beta"], 0, path="large")
        ns.alloc(C2)
        n = pta.n
        z = np.zeros((C2, n))
        z[:, ::17] = 1.0
        al = np.where(z > 0, 25.0, 1.0)
        ns.set_state(x=x, z=z, alpha=al, theta=np.full(C2, 0.05), nu=np.full(C2, 4.0))
        _, h = ns.eval_lnlike()
        ns.close()
        orc = Oracle(pta, OutlierModel(**MODELS["beta"]))
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            for k in range(C2):
                st = ChainState(b=np.zeros(pta.m), z=z[k], alpha=al[k], pout=np.zeros(n),
                                theta=0.05, nu=4.0)
                orc.cache = None
                want64 = orc.lnlike_marginal(st, x[k])
                ext = lnlike_marginal_extended(pta, st, x[k])
                tol = max(1e-9 * abs(ext), 4 * abs(want64 - ext))
                assert abs(h[k] - ext) <= tol, (overlap, k, h[k], ext, want64)


@pytest.mark.parametrize("name", ["ebig_beta_fixed", "ebig_t_fixed", "mb_beta_fixed",
                                  "mb_t_fixed", "mbn_vvh17_fixed"])
def test_register_epochs_first_matches_lds_epochs_first(name):
    """lg_hyper_ecr (round 6: the epochs-first elimination on one wave per chain, register-
    resident 8x8-cyclic factor, the epochs' rank-1 downdates on the VALU) against lg_hyper<2>
    (256 threads, LDS, MFMA rank update; GST_DEBUG_EPOCHS_LDS): the same elimination order
    [ECORR | TM | Fourier] and Philox normals, so the b-marginalised likelihood agrees to
    1e-10 at 256 states (prior draws, the fixture's latents) and 16 chains x 6 sweeps from
    the fixture's start make the same MH, z and nu decisions with b, alpha, pout, theta within
    1e-8 relative."""
    _compare_large_variants(name, {}, {"epochs_lds": True})


@pytest.mark.parametrize("name", ["ebig_beta_fixed", "ebig_t_fixed", "mb_beta_fixed",
                                  "mb_t_fixed", "mbn_vvh17_fixed"])
def test_structured_ecorr_gram_matches_dense_gram(name):
    """lg_gram_ec (round 6: for disjoint ECORR epochs run epochs first, only G_xx, the epochs'
    diagonal and their couplings to [timing model | Fourier | r], by MFMA over the compact
    columns and over the epoch-ordered TOAs) against the dense Gram (GST_DEBUG_LARGE_GRAM:
    lg_gram / lg_gram_small over all mp columns): the same hyper kernel on Grams that differ
    in summation order only, held to the tolerances of the two eliminations above."""
    _compare_large_variants(name, {}, {"large_gram": True})


def _compare_large_variants(name, dbg_a, dbg_b):
    """Likelihoods at 256 states and 16 chains x 6 sweeps of two large-path builds of the same
    chain (debug flags dbg_a, dbg_b) from the fixture's start."""
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    from golden_io import load_ref, sweep_state
    ref = load_ref(name)
    pta = ref["pta"]
    s0 = sweep_state(ref, 0)
    C2 = 256
    lo = np.array([p.pmin for p in pta.params])
    hi = np.array([p.pmax for p in pta.params])
    x = np.random.default_rng(12).uniform(lo, hi, size=(C2, len(lo)))
    got, outs = [], []
    for dbg in (dbg_a, dbg_b):
        ns = NativeSampler(pta, ref["kw"], 0, path="large")
        ns.set_debug(**dbg)
        ns.alloc(C2)
        ns.set_state(x=x, b=np.tile(s0["b"], (C2, 1)), z=np.tile(s0["z"], (C2, 1)),
                     alpha=np.tile(s0["alpha"], (C2, 1)), pout=np.tile(s0["pout"], (C2, 1)),
                     theta=np.full(C2, s0["theta"]), nu=np.full(C2, s0["nu"]))
        got.append(ns.eval_lnlike())
        ns.close()
        ns = NativeSampler(pta, ref["kw"], 0, path="large")
        ns.set_debug(**dbg)
        ns.alloc(C)
        ns.set_state(x=np.tile(ref["xs"], (C, 1)), b=np.tile(s0["b"], (C, 1)),
                     z=np.tile(s0["z"], (C, 1)), alpha=np.tile(s0["alpha"], (C, 1)),
                     pout=np.tile(s0["pout"], (C, 1)), theta=np.full(C, s0["theta"]),
                     nu=np.full(C, s0["nu"]))
        rec = ns.alloc_records(S)
        ns.sweep(S, records=rec, seed=35)
        out = {k: v.cpu().numpy() for k, v in rec.items()}
        out["status"] = ns.get_state()["status"]
        ns.close()
        outs.append(out)
    (w1, h1), (w2, h2) = got
    np.testing.assert_array_equal(w1, w2)
    ok = np.isfinite(h2)
    assert ok.sum() > C2 // 2
    np.testing.assert_array_equal(np.isfinite(h1), ok)
    r = np.abs(h1[ok] - h2[ok]) / np.abs(h2[ok])
    assert r.max() <= 1e-10, r.max()
    a, b = outs
    assert np.all((a["status"] & STATUS_ERRORS) == 0)
    np.testing.assert_array_equal(a["status"], b["status"])
    for k in ("x", "z", "nu"):
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
    eb = np.linalg.norm(a["b"] - b["b"], axis=-1) / np.maximum(np.linalg.norm(b["b"], axis=-1),
                                                                1e-300)
    assert np.all(eb <= 1e-8), ("b", eb.max())
    # (pout is a probability: within 1e-8 relative or 1e-9 absolute -- vvh17's Sigma reaches
    # cond ~ 1e22, where the two eliminations' b draws differ by cond x eps in the directions
    # the data leave free, which moves the small pout values of the flagged TOAs at 1e-10)
    for k in ("alpha", "pout", "theta"):
        d = np.abs(a[k] - b[k])
        tol = 1e-8 * np.maximum(np.abs(b[k]), 1e-300) + (1e-9 if k == "pout" else 1e-300)
        assert np.all(d <= tol), (k, d.max())
