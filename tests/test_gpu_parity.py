"""HIP path vs the reference (golden fixtures from tools/gen_golden.py), injected variates.

Tolerances (north star): continuous outputs <= 1e-10 relative (fp64); discrete draws --
MH accept/reject (hence x), z, nu -- exactly equal.  The b draw is compared with the
reference's own Cholesky mean cho_solve(Sigma, d) (gibbs.py:321-322) plus the reference's
draw term U S^-1/2 xi (gibbs.py:169-180): its SVD mean is inaccurate when cond(Sigma) is
large (SURVEY.md 8a R6 parity note), so it is used only for well-conditioned sweeps.
"""
import numpy as np
import pytest

from golden_io import fixture_names, load_ref, oracle_replay, sweep_state

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a HIP device", allow_module_level=True)

from gibbs_student_t_amd._abi import STATUS_ERRORS, STATUS_FLOOR  # noqa: E402
from gibbs_student_t_amd import _abi  # noqa: E402
from gibbs_student_t_amd.native import NativeSampler, pack_tape  # noqa: E402
import scipy.linalg as sl  # noqa: E402

from oracle.gibbs_oracle import (ChainState, Oracle, OutlierModel,  # noqa: E402
                                 b_mean_extended, lnlike_marginal_extended)

NAMES = fixture_names()
RTOL = 1e-10


PATHS = ("persistent", "large")


def _native(ref, C, path="auto"):
    try:
        ns = NativeSampler(ref["pta"], ref["kw"], 0, path=path)
    except _abi.GstNativeError as e:
        # the persistent kernel's instances (gst_shapes.h) do not cover this model: its
        # parity runs on the large path only (test_general_white_noise_path_choice pins which)
        if path == "persistent" and "no persistent-kernel instance" in str(e):
            pytest.skip("beyond the persistent kernel's shapes (large path only)")
        raise
    assert path == "auto" or ns.path == path
    ns.alloc(C)
    return ns


@pytest.mark.parametrize("name", [n for n in NAMES
                                  if n.startswith(("ecb", "ecn", "ecq", "ebig", "mb", "jb"))])
def test_general_white_noise_path_choice(name):
    """Per-backend efac / equad and ECORR models (gibbs.py:64-77) run on the persistent
    kernel's general white-noise instances when their hyper block fits (ecb / ecn: 20 Fourier +
    24 ECORR columns; jb: J1713+0747 with per-backend efac / equad, 60 Fourier columns and
    n = 130 on the three-slot instance), on the large path otherwise (mb / mbn: 80 columns;
    ebig: 150)."""
    ref = load_ref(name)
    ns = NativeSampler(ref["pta"], ref["kw"], 0)
    assert ns.path == ("persistent" if name.startswith(("ecb", "ecn", "ecq", "jb")) else "large")
    if ns.path == "persistent":
        # two waves per chain (round 6: the general white-noise instances have the pair build;
        # bitwise equality with one wave is test_gpu_waves.py's): forced and automatic both run
        ns.alloc(8)
        s0 = sweep_state(ref, 0)
        ns.set_state(x=np.tile(ref["chain"][0], (8, 1)), b=np.tile(s0["b"], (8, 1)),
                     z=np.tile(s0["z"], (8, 1)), alpha=np.tile(s0["alpha"], (8, 1)),
                     pout=np.tile(s0["pout"], (8, 1)), theta=np.full(8, s0["theta"]),
                     nu=np.full(8, s0["nu"]))
        ns.set_waves(2)
        ns.sweep(1, seed=1)
        ns.set_waves("auto")
        ns.sweep(1, seed=1, sweep0=1)
        assert np.all((ns.get_state()["status"] & _abi.STATUS_ERRORS) == 0)
    ns.close()


def _rel(a, b):
    a, b = np.asarray(a, float), np.asarray(b, float)
    both_inf = np.isinf(a) & np.isinf(b) & (np.sign(a) == np.sign(b))
    d = np.where(both_inf, 0.0, np.abs(a - b) / np.maximum(np.abs(b), 1e-300))
    return d


def _states(ref, idx):
    ss = [sweep_state(ref, i) for i in idx]
    return {k: np.stack([s[k] for s in ss]) for k in ("b", "z", "alpha", "pout")}, ss


@pytest.mark.parametrize("name", NAMES)
@pytest.mark.parametrize("path", PATHS)
def test_lnlikelihoods(name, path):
    """get_lnlikelihood_white / get_lnlikelihood at every point the reference evaluated."""
    ref = load_ref(name)
    tape = ref["tape"]
    S = int(ref["niter"])
    for which, K in (("white", 21), ("hyper", 11)):
        idx = np.repeat(np.arange(S), K)
        st, ss = _states(ref, idx)
        xs = tape[f"{which}_lnl_x"].reshape(S * K, -1)
        want = tape[f"{which}_lnl"].reshape(-1)
        ns = _native(ref, S * K, path)
        ns.set_state(x=xs, theta=np.array([s["theta"] for s in ss]),
                     nu=np.array([s["nu"] for s in ss]), **st)
        w, h = ns.eval_lnlike()
        got = w if which == "white" else h
        r = _rel(got, want)
        bad = np.flatnonzero(r > RTOL)
        for k in bad:
            # ill-conditioned Sigma: the reference's own fp64 value is inexact.  Arbitrate
            # with the long-double value: the GPU error must be within twice the
            # reference's own error, or within 1e-10 of the magnitude of the cancelling
            # terms (log|N|, r^T N^-1 r, d^T Sigma^-1 d, log|Sigma|, log|phi|)
            s = ss[k]
            st_k = ChainState(b=s["b"], z=s["z"], alpha=s["alpha"], pout=s["pout"],
                              theta=s["theta"], nu=s["nu"])
            assert which == "hyper", f"white lnL mismatch {r[k]:.3e} at {k}"
            ext, scale = lnlike_marginal_extended(ref["pta"], st_k, xs[k], with_scale=True)
            err = abs(got[k] - ext)
            assert err <= max(2 * abs(want[k] - ext), RTOL * scale), \
                f"{which}[{k}]: gpu {got[k]!r} ref {want[k]!r} extended {ext!r} scale {scale:.3e}"
        ns.close()


@pytest.mark.parametrize("name", NAMES)
@pytest.mark.parametrize("path", PATHS)
def test_mh_blocks_and_b_draw(name, path):
    """White MH + Gram + hyper MH + b draw, each sweep from the reference's start state."""
    ref = load_ref(name)
    S = int(ref["niter"])
    idx = np.arange(S)
    st, ss = _states(ref, idx)
    ns = _native(ref, S, path)
    ns.set_state(x=ref["chain"][:S], theta=np.array([s["theta"] for s in ss]),
                 nu=np.array([s["nu"] for s in ss]), **st)
    rows = pack_tape(ref["tape"], idx, ns.n, ns.m, ns.stride)
    tape = torch.as_tensor(rows[:, None, :]).to(ns.tdev).contiguous()
    ns.sweep(1, mask=_abi.STAGE_WHITE | _abi.STAGE_HYPER | _abi.STAGE_B, tape=tape)
    out = ns.get_state()
    assert np.all((out["status"] & _abi.STATUS_ERRORS) == 0)
    # x after the hyper block == the next sweep's recorded x: exact (same MH decisions)
    np.testing.assert_array_equal(out["x"][:S - 1], ref["chain"][1:S])
    t = ref["tape"]
    drew = ~np.isnan(t["b_cond"])
    want = t["b_mean_chol"] + t["b_delta"]
    orc = Oracle(ref["pta"], OutlierModel(**ref["kw"]))
    for i in np.flatnonzero(drew):
        s = ss[i]
        st_i = ChainState(b=s["b"], z=s["z"], alpha=s["alpha"], pout=s["pout"],
                          theta=s["theta"], nu=s["nu"])
        x_h = ref["chain"][i + 1] if i + 1 < S else out["x"][i]
        orc.cache = None
        Sigma, d = orc.sigma_matrix(st_i, x_h)
        f = orc.floor_shift(Sigma)
        # the SVD noise floor (Sigma beyond fp64 resolution): flagged and counted, and b is
        # the exact draw from Sigma + f I -- the oracle's floor mean plus the reference's
        # draw term; only vvh17 fixtures (alpha = 1e10 on flagged TOAs) reach the gate
        assert bool(out["status"][i] & _abi.STATUS_FLOOR) == (f > 0.0), f"sweep {i}: f {f:.3e}"
        assert int(_abi.floor_draws(out["status"][i])) == (1 if f > 0.0 else 0)
        assert f == 0.0 or "vvh17" in name, f"sweep {i}: floor gate on a non-vvh17 fixture"
        if f > 0.0:
            wf = sl.cho_solve(sl.cho_factor(Sigma + f * np.eye(len(d))), d) + t["b_delta"][i]
            err = np.linalg.norm(out["b"][i] - wf) / np.linalg.norm(wf)
            assert err <= 1e-9, f"sweep {i}: floor b err {err:.3e}"
            assert_floor_draw_within_reference_error(out["b"][i], t, i, Sigma, d, f)
            continue
        err = np.linalg.norm(out["b"][i] - want[i]) / np.linalg.norm(want[i])
        if err > 1e-9:
            # cond(Sigma) so large that fp64 Cholesky means (LAPACK's and ours) both carry
            # ~cond*eps error: arbitrate with the long-double mean, allowing twice the
            # reference's own error
            mext = b_mean_extended(ref["pta"], st_i, x_h)
            e_gpu = np.linalg.norm(out["b"][i] - (mext + t["b_delta"][i]))
            e_ref = np.linalg.norm(t["b_mean_chol"][i] - mext)
            assert e_gpu <= 2 * e_ref + 1e-12 * np.linalg.norm(mext), \
                f"sweep {i}: b err {err:.3e} (cond {t['b_cond'][i]:.2e}), " \
                f"vs extended {e_gpu:.3e} > 2 x ref {e_ref:.3e}"
        if t["b_cond"][i] < 1e7:
            err_svd = np.linalg.norm(out["b"][i] - t["b_ref"][i]) / np.linalg.norm(t["b_ref"][i])
            assert err_svd <= 1e-9
    for i in np.flatnonzero(~drew):
        np.testing.assert_array_equal(out["b"][i], ref["bchain"][i])


def assert_floor_draw_within_reference_error(b_gpu, t, i, Sigma, d, f):
    """A b draw at the SVD noise floor against the reference's OWN b (``b_ref``, its SVD draw
    u (u^T d / s) + U S^-1/2 xi, gibbs.py:166-180) on the same sweep: the GPU b must be no
    further from it than the exact draw (cho_solve(Sigma, d) + the same draw term) is, or the
    shift f I must lie within the reference's own SVD error -- the perturbation
    ||U S U^T - Sigma||_2 that LAPACK's SVD itself makes of Sigma on this sweep (long-double
    reconstruction of the recomputed SVD, which must be bitwise the fixture's)."""
    b_ref = t["b_ref"][i]
    e_gpu = np.linalg.norm(b_gpu - b_ref)
    e_exact = np.linalg.norm(t["b_mean_chol"][i] + t["b_delta"][i] - b_ref)
    if e_gpu <= e_exact:
        return
    u, sv, _ = sl.svd(Sigma)
    np.testing.assert_array_equal(u @ ((u.T @ d) / sv), t["b_mean_svd"][i])
    ld = np.longdouble
    E = (u.astype(ld) * sv.astype(ld)) @ u.T.astype(ld) - Sigma.astype(ld)
    e_svd = np.linalg.norm(E.astype(np.float64), 2)
    assert f <= e_svd, (f"sweep {i}: floor b {e_gpu:.3e} from the reference's b (exact draw "
                        f"{e_exact:.3e}) and f {f:.3e} > the SVD's own error {e_svd:.3e}")


@pytest.mark.parametrize("name", NAMES)
@pytest.mark.parametrize("path", PATHS)
def test_outlier_stages(name, path):
    """theta, z, alpha, nu from the reference's post-b state (gibbs.py:377-380)."""
    ref = load_ref(name)
    S = int(ref["niter"]) - 1
    idx = np.arange(S)
    pre = [sweep_state(ref, i) for i in idx]
    post = [sweep_state(ref, i + 1) for i in idx]
    ns = _native(ref, S, path)
    ns.set_state(x=ref["chain"][1:S + 1], b=np.stack([s["b"] for s in post]),
                 z=np.stack([s["z"] for s in pre]), alpha=np.stack([s["alpha"] for s in pre]),
                 pout=np.stack([s["pout"] for s in pre]),
                 theta=np.array([s["theta"] for s in pre]), nu=np.array([s["nu"] for s in pre]))
    rows = pack_tape(ref["tape"], idx, ns.n, ns.m, ns.stride)
    tape = torch.as_tensor(rows[:, None, :]).to(ns.tdev).contiguous()
    ns.sweep(1, mask=_abi.STAGE_THETA | _abi.STAGE_Z | _abi.STAGE_ALPHA | _abi.STAGE_DF,
             tape=tape)
    out = ns.get_state()
    want = {k: np.stack([np.asarray(s[k], float) for s in post]) for k in
            ("z", "alpha", "pout", "theta", "nu")}
    np.testing.assert_array_equal(out["z"], want["z"])
    np.testing.assert_array_equal(out["nu"], want["nu"])
    np.testing.assert_array_equal(out["theta"], want["theta"])
    for k in ("alpha", "pout"):
        r = _rel(out[k], want[k])
        assert np.all(r <= RTOL), f"{k}: max rel {r.max():.3e}"


@pytest.mark.parametrize("name", [n for n in NAMES if "fixed" in n and "vvh17" not in n])
@pytest.mark.parametrize("path", PATHS)
def test_full_chain_replay(name, path):
    """12 consecutive sweeps of one chain on the reference's tape (gibbs.py:342-385),
    against the reference's OWN chain: discrete draws exact; the continuous records carry
    the reference's SVD-mean error compounded over the sweeps, hence
    max(1e-6, eps x the largest cond(Sigma) of the replay) here -- b normwise per sweep,
    alpha / pout / theta elementwise.  ECORR models reach cond ~ 2e13, where the reference's
    own chain is ~1e-4 from the exact algorithm's (0.2 eps cond at most over every fixture,
    measured with the oracle).  The 1e-10 check of the same replay is
    test_full_chain_replay_vs_oracle."""
    ref = load_ref(name)
    S = int(ref["niter"])
    s0 = sweep_state(ref, 0)
    ns = _native(ref, 1, path)
    ns.set_state(x=ref["xs"][None], b=s0["b"][None], z=s0["z"][None],
                 alpha=s0["alpha"][None], pout=s0["pout"][None], theta=np.array([s0["theta"]]),
                 nu=np.array([s0["nu"]]))
    rows = pack_tape(ref["tape"], np.arange(S), ns.n, ns.m, ns.stride)
    tape = torch.as_tensor(rows[None]).to(ns.tdev).contiguous()
    rec = ns.alloc_records(S)
    ns.sweep(S, records=rec, tape=tape)
    got = {k: v.cpu().numpy()[0] for k, v in rec.items()}
    np.testing.assert_array_equal(got["x"], ref["chain"])
    np.testing.assert_array_equal(got["z"], ref["zchain"])
    np.testing.assert_array_equal(got["nu"], ref["dfchain"])
    tol = max(1e-6, np.finfo(float).eps * np.nanmax(ref["tape"]["b_cond"]))
    nb = np.linalg.norm(ref["bchain"], axis=1)
    eb = np.linalg.norm(got["b"] - ref["bchain"], axis=1) / np.where(nb > 0, nb, 1.0)
    assert np.all(eb <= tol), f"b: max normwise rel {eb.max():.3e} > {tol:.1e}"
    for k, rk in (("alpha", "alphachain"), ("pout", "poutchain"), ("theta", "thetachain")):
        r = _rel(got[k], ref[rk])
        assert np.all(r <= tol), f"{k}: max rel {r.max():.3e} > {tol:.1e}"


def assert_replay_matches(got, want, ref, label=""):
    """Discrete records exact; b normwise per sweep, alpha / pout elementwise <= RTOL.

    Where the two fp64 Cholesky means (LAPACK's in the oracle, the kernel's) differ by more
    than RTOL -- cond(Sigma) ~ 1e8 leaves both ~1e-10 from the exact mean -- the long-double
    mean arbitrates, as in test_mh_blocks_and_b_draw: the GPU b must then be at least as
    close to it as the oracle's (within twice its error)."""
    n = want["z"].shape[-1]
    for k in ("x", "z", "nu", "theta"):
        g = got[k][..., :n] if k == "z" else got[k]
        np.testing.assert_array_equal(g, want[k], err_msg=f"{label} {k}")
    eb = np.linalg.norm(got["b"] - want["b"], axis=1) / np.maximum(
        np.linalg.norm(want["b"], axis=1), 1e-300)
    delta = ref["tape"]["b_delta"]
    orc = Oracle(ref["pta"], OutlierModel(**ref["kw"]))
    for k in np.flatnonzero(eb > RTOL):
        assert k >= 1, f"{label} b differs at the start state"
        # b recorded at sweep k was drawn in sweep k-1 at that sweep's (z, alpha) and x_k
        st = ChainState(b=want["b"][k - 1], z=want["z"][k - 1], alpha=want["alpha"][k - 1],
                        pout=want["pout"][k - 1], theta=float(want["theta"][k - 1]),
                        nu=float(want["nu"][k - 1]))
        orc.cache = None
        f = orc.floor_shift(orc.sigma_matrix(st, want["x"][k])[0])   # the draw's floor shift
        exact = b_mean_extended(ref["pta"], st, want["x"][k], shift=f) + delta[k - 1]
        e_gpu = np.linalg.norm(got["b"][k] - exact)
        e_orc = np.linalg.norm(want["b"][k] - exact)
        assert e_gpu <= 2 * e_orc + 1e-13 * np.linalg.norm(exact), \
            f"{label} b sweep {k}: rel {eb[k]:.3e}, |gpu - exact| {e_gpu:.3e} > " \
            f"2 |oracle - exact| {e_orc:.3e}"
    for k in ("alpha", "pout"):
        r = _rel(got[k][..., :n], want[k])
        assert np.all(r <= RTOL), f"{label} {k}: max rel {r.max():.3e}"


@pytest.mark.parametrize("name", [n for n in NAMES if "fixed" in n])
@pytest.mark.parametrize("path", PATHS)
def test_full_chain_replay_vs_oracle(name, path):
    """12 consecutive sweeps on the reference's tape against the oracle replaying the
    same tape with the Cholesky-mean b draw (at the SVD noise floor: the mean of Sigma + f I,
    Oracle.floor_shift -- the vvh17 fixtures): discrete draws exact, every continuous record
    <= 1e-10 relative (b normwise per sweep, alpha / pout / theta elementwise)."""
    ref = load_ref(name)
    S = int(ref["niter"])
    s0 = sweep_state(ref, 0)
    ns = _native(ref, 1, path)
    ns.set_state(x=ref["xs"][None], b=s0["b"][None], z=s0["z"][None],
                 alpha=s0["alpha"][None], pout=s0["pout"][None], theta=np.array([s0["theta"]]),
                 nu=np.array([s0["nu"]]))
    rows = pack_tape(ref["tape"], np.arange(S), ns.n, ns.m, ns.stride)
    tape = torch.as_tensor(rows[None]).to(ns.tdev).contiguous()
    rec = ns.alloc_records(S)
    ns.sweep(S, records=rec, tape=tape)
    got = {k: v.cpu().numpy()[0] for k, v in rec.items()}
    ns.close()
    assert_replay_matches(got, oracle_replay(ref, S), ref, name)


@pytest.mark.parametrize("path", PATHS)
def test_failed_factor_never_draws_b(path):
    """Sigma not positive definite at the hyper block's start (negative noise weights) and
    every proposal out of the prior: no factor exists to draw b from, so the chain keeps
    its b and flags status 2 (gibbs.py:320-324 gives -inf; it never reaches a b draw)."""
    ref = load_ref("beta_fixed")
    s0 = sweep_state(ref, 0)
    ns = _native(ref, 1, path)
    alpha = np.full_like(s0["alpha"], -1.0)            # N = alpha^z N0 < 0 where z = 1
    b0 = np.linspace(-1e-7, 1e-7, ns.m)[None]
    ns.set_state(x=ref["xs"][None], b=b0, z=np.ones_like(s0["z"])[None], alpha=alpha[None],
                 pout=s0["pout"][None], theta=np.array([s0["theta"]]),
                 nu=np.array([s0["nu"]]))
    rows = pack_tape(ref["tape"], [0], ns.n, ns.m, ns.stride)
    for step in range(10):
        rows[0, _abi.TAPE_HYPER + 4 * step + 2] = 1e6     # jump far outside the prior box
    tape = torch.as_tensor(rows[:, None, :]).to(ns.tdev).contiguous()
    ns.sweep(1, mask=_abi.STAGE_HYPER | _abi.STAGE_B | _abi.STAGE_B_FORCE, tape=tape)
    out = ns.get_state()
    assert out["status"][0] & 2 and out["status"][0] & 1
    np.testing.assert_array_equal(out["b"], b0)
    np.testing.assert_array_equal(out["x"][0], ref["xs"])
    ns.close()


@pytest.mark.parametrize("path", PATHS)
def test_philox_mode_runs_and_moves(path):
    ref = load_ref("beta_fixed")
    C, S = 256, 50
    ns = _native(ref, C, path)
    s0 = sweep_state(ref, 0)
    ns.set_state(x=np.tile(ref["xs"], (C, 1)), b=np.tile(s0["b"], (C, 1)),
                 z=np.tile(s0["z"], (C, 1)), alpha=np.tile(s0["alpha"], (C, 1)),
                 pout=np.tile(s0["pout"], (C, 1)), theta=np.full(C, s0["theta"]),
                 nu=np.full(C, s0["nu"]))
    rec = ns.alloc_records(S)
    ns.sweep(S, records=rec, seed=1234)
    x = rec["x"].cpu().numpy()
    out = ns.get_state()
    assert np.all(np.isfinite(x)) and np.all(np.isfinite(out["b"]))
    assert np.all((out["status"] & STATUS_ERRORS) == 0)
    # chains decorrelate from the common start
    assert np.std(x[:, -1, :], axis=0).min() > 0
    names = ref["pta"].param_names
    lo = np.array([p.pmin for p in ref["pta"].params])
    hi = np.array([p.pmax for p in ref["pta"].params])
    assert np.all((x >= lo) & (x <= hi)), names


@pytest.mark.parametrize("path", PATHS)
def test_sharding_invariance(path):
    """Chains keyed by global id: one launch of C == two launches of C/2 (bitwise)."""
    ref = load_ref("uniform_prior")
    C, S = 16, 5
    s0 = sweep_state(ref, 0)
    init = dict(x=np.tile(ref["xs"], (C, 1)), b=np.tile(s0["b"], (C, 1)),
                z=np.tile(s0["z"], (C, 1)), alpha=np.tile(s0["alpha"], (C, 1)),
                pout=np.tile(s0["pout"], (C, 1)), theta=np.full(C, s0["theta"]),
                nu=np.full(C, s0["nu"]))
    ns = _native(ref, C, path)
    ns.set_state(**init)
    ns.sweep(S, seed=99, sweep0=7)
    full = ns.get_state()
    halves = []
    for h in range(2):
        nh = _native(ref, C // 2, path)
        nh.set_state(**{k: v[h * C // 2:(h + 1) * C // 2] for k, v in init.items()})
        nh.sweep(S, seed=99, sweep0=7, chain0=h * C // 2)
        halves.append(nh.get_state())
    for k in ("x", "b", "z", "alpha", "pout", "theta", "nu"):
        np.testing.assert_array_equal(full[k], np.concatenate([h[k] for h in halves]))


def test_two_chains_per_simd_build_matches():
    """A launch with more chains than SIMDs runs the 256-register (two chains per SIMD)
    build; it must give bitwise the chains of the uncapped build (two half launches)."""
    ref = load_ref("beta_prior")
    C, S = 2048, 8
    s0 = sweep_state(ref, 0)
    lo = np.array([p.pmin for p in ref["pta"].params])
    hi = np.array([p.pmax for p in ref["pta"].params])
    init = dict(x=np.random.default_rng(11).uniform(lo, hi, size=(C, len(lo))),
                b=np.tile(s0["b"], (C, 1)), z=np.tile(s0["z"], (C, 1)),
                alpha=np.tile(s0["alpha"], (C, 1)), pout=np.tile(s0["pout"], (C, 1)),
                theta=np.full(C, s0["theta"]), nu=np.full(C, s0["nu"]))
    ns = _native(ref, C, "persistent")
    ns.set_state(**init)
    rec = ns.alloc_records(S)
    ns.sweep(S, records=rec, seed=21, sweep0=4)
    full = ns.get_state()
    frec = {k: v.cpu().numpy() for k, v in rec.items()}
    ns.close()
    for h in range(2):
        sl = slice(h * C // 2, (h + 1) * C // 2)
        nh = _native(ref, C // 2, "persistent")
        nh.set_state(**{k: v[sl] for k, v in init.items()})
        hrec = nh.alloc_records(S)
        nh.sweep(S, records=hrec, seed=21, sweep0=4, chain0=h * C // 2)
        half = nh.get_state()
        for k in ("x", "b", "z", "alpha", "pout", "theta", "nu", "status"):
            np.testing.assert_array_equal(full[k][sl], half[k], err_msg=k)
        for k, v in hrec.items():
            np.testing.assert_array_equal(frec[k][sl], v.cpu().numpy(), err_msg=f"rec {k}")
        nh.close()


def test_paths_agree_in_philox_mode():
    """Both paths draw the same Philox variates: J1713 chains follow the same MH/z/nu
    decisions (floating-point differences are ~1e-13, far from any decision threshold)."""
    ref = load_ref("beta_prior")
    C, S = 64, 6
    s0 = sweep_state(ref, 0)
    lo = np.array([p.pmin for p in ref["pta"].params])
    hi = np.array([p.pmax for p in ref["pta"].params])
    init = dict(x=np.random.default_rng(3).uniform(lo, hi, size=(C, len(lo))),
                b=np.tile(s0["b"], (C, 1)), z=np.tile(s0["z"], (C, 1)),
                alpha=np.tile(s0["alpha"], (C, 1)), pout=np.tile(s0["pout"], (C, 1)),
                theta=np.full(C, s0["theta"]), nu=np.full(C, s0["nu"]))
    out = {}
    for path in PATHS:
        ns = _native(ref, C, path)
        ns.set_state(**init)
        ns.sweep(S, seed=5, sweep0=2)
        out[path] = ns.get_state()
        ns.close()
    a, b = out["persistent"], out["large"]
    same = np.all(a["x"] == b["x"], axis=1) & np.all(a["z"] == b["z"], axis=1) & \
        (a["nu"] == b["nu"])
    assert same.mean() >= 0.95, same.mean()
    for k in ("b", "alpha", "pout", "theta"):
        r = _rel(b[k][same], a[k][same])
        assert np.all(r <= 1e-8), f"{k}: max rel {r.max():.3e}"


@pytest.mark.parametrize("name,path", [("c20_beta_fixed", "persistent"),
                                       ("tm22_beta_fixed", "persistent"),
                                       ("beta_fixed", "persistent"),
                                       ("scaled_beta_fixed", "large")])
def test_auto_path_choice(name, path):
    """Register-resident instances cover <= 20 components (MT 8), <= 30 with <= 16 TM
    columns and <= 26 with 17..24 TM columns (MT 10), padded with unit-prior dummies;
    larger models take the large path."""
    ref = load_ref(name)
    ns = NativeSampler(ref["pta"], ref["kw"], 0)
    assert ns.path == path
    ns.close()
