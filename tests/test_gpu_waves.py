"""Two waves per chain (gst_set_waves) and the b record after a sweep
that skips the b draw (gibbs.py:373).

The two-wave kernel splits the red-noise MH block's likelihood evaluations between the
chain's two waves (the next proposal, and the one after it on the reject branch), then
replays the reference's decisions (gibbs.py:99-110) on the exchanged values, so its chains
must be BITWISE those of the one-wave kernel: same variates, same decisions, the b draw
from a factor of the same point computed by the same code."""
import numpy as np
import pytest

from gibbs_student_t_amd import _abi

from golden_io import load_ref, sweep_state
from test_gpu_parity import PATHS, _native

pytestmark = pytest.mark.gpu

KEYS = ("x", "b", "z", "alpha", "pout", "theta", "nu")


def _init(ref, C, seed):
    s0 = sweep_state(ref, 0)
    lo = np.array([p.pmin for p in ref["pta"].params])
    hi = np.array([p.pmax for p in ref["pta"].params])
    return dict(x=np.random.default_rng(seed).uniform(lo, hi, size=(C, len(lo))),
                b=np.tile(s0["b"], (C, 1)), z=np.tile(s0["z"], (C, 1)),
                alpha=np.tile(s0["alpha"], (C, 1)), pout=np.tile(s0["pout"], (C, 1)),
                theta=np.full(C, s0["theta"]), nu=np.full(C, s0["nu"]))


def _run(ref, C, S, waves, init, mask=_abi.STAGE_ALL, seed=7, sweep0=3, chain0=0):
    ns = _native(ref, C, "persistent")
    ns.set_waves(waves)
    ns.set_state(**init)
    rec = ns.alloc_records(S)
    ns.sweep(S, records=rec, seed=seed, sweep0=sweep0, mask=mask, chain0=chain0)
    out = ns.get_state()
    recs = {k: v.cpu().numpy() for k, v in rec.items()}
    ns.close()
    return out, recs


# every model family, the efac-varied fixture, the 5%-outlier simulate_data pulsar, and
# the two other register shapes (20 components: MT = 8; 22 timing-model columns: K0 = 3)
FIXTURES = ("beta_prior", "t_prior", "gaussian_prior", "uniform_prior", "vvh17_prior",
            "beta_efac_fixed", "c3_beta_fixed", "c20_t_fixed", "tm22_beta_fixed",
            # the general white-noise instances (round 6): two backends + ECORR, one backend +
            # ECORR, J1713+0747 with two backends
            "ecb_beta_fixed", "ecq_t_fixed", "jb_uniform_fixed")


@pytest.mark.parametrize("name", FIXTURES)
def test_two_waves_match_one_wave(name):
    ref = load_ref(name)
    C, S = 96, 24
    init = _init(ref, C, 5)
    one, r1 = _run(ref, C, S, 1, init)
    two, r2 = _run(ref, C, S, 2, init)
    for k in KEYS + ("status",):
        np.testing.assert_array_equal(one[k], two[k], err_msg=k)
    for k in KEYS:
        np.testing.assert_array_equal(r1[k], r2[k], err_msg=f"rec {k}")


@pytest.mark.parametrize("mask", [_abi.STAGE_HYPER | _abi.STAGE_B,
                                  _abi.STAGE_B | _abi.STAGE_B_FORCE,
                                  _abi.STAGE_HYPER,
                                  _abi.STAGE_ALL & ~_abi.STAGE_HYPER,
                                  _abi.STAGE_Z, _abi.STAGE_ALPHA,
                                  _abi.STAGE_Z | _abi.STAGE_ALPHA])
def test_two_waves_stage_masks(mask):
    """The drop-in's update_* methods launch stage subsets; each subset must agree too --
    also multi-sweep launches of the z / alpha stages alone, where no other stage's barrier
    separates one sweep's LDS exchange from the next."""
    ref = load_ref("beta_prior")
    C, S = 64, 6
    init = _init(ref, C, 9)
    one, r1 = _run(ref, C, S, 1, init, mask=mask)
    two, r2 = _run(ref, C, S, 2, init, mask=mask)
    for k in KEYS + ("status",):
        np.testing.assert_array_equal(one[k], two[k], err_msg=k)


def test_auto_waves_choice():
    """AUTO runs two waves per chain up to 2 x CUs chains: 512 chains (config 3) then match
    the forced one-wave kernel bitwise."""
    ref = load_ref("c3_beta_fixed")
    C, S = 512, 5
    init = _init(ref, C, 13)
    auto, ra = _run(ref, C, S, "auto", init)
    one, r1 = _run(ref, C, S, 1, init)
    for k in KEYS + ("status",):
        np.testing.assert_array_equal(auto[k], one[k], err_msg=k)


@pytest.mark.parametrize("path,waves", [(p, 1) for p in PATHS] + [("persistent", 2)])
def test_b_record_after_skipped_draw(path, waves):
    """gibbs.py:373 skips the b draw unless every parameter differs from chain[ii, -1] (the
    white-noise equad on J1713).  With the white block off the equad never moves, so every
    sweep skips the draw: every b record, and the final b, must be the initial b exactly
    (the red-noise block still runs and reuses the LDS the b vector is staged in)."""
    ref = load_ref("beta_prior")
    C, S = 128, 40
    init = _init(ref, C, 17)
    ns = _native(ref, C, path)
    if path == "persistent":
        ns.set_waves(waves)
    ns.set_state(**init)
    rec = ns.alloc_records(S)
    ns.sweep(S, records=rec, seed=3, sweep0=0, mask=_abi.STAGE_ALL & ~_abi.STAGE_WHITE)
    x = rec["x"].cpu().numpy()
    b = rec["b"].cpu().numpy()
    fin = ns.get_state()
    ns.close()
    assert np.any(x[:, 1:, :2] != x[:, :1, :2])           # the red-noise block moved
    np.testing.assert_array_equal(x[:, :, -1], np.repeat(init["x"][:, -1:], S, axis=1))
    np.testing.assert_array_equal(b, np.repeat(init["b"][:, None], S, axis=1))
    np.testing.assert_array_equal(fin["b"], init["b"])
