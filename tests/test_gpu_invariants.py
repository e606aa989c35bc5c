"""Launch-boundary invariants of the persistent kernel: no hidden cross-sweep state.

A chain's state between sweeps is, by the reference's semantics (gibbs.py:354-380), exactly
(x, b, z, alpha, pout, theta, nu) -- what the records hold.  The persistent kernel keeps
more than that across the sweeps of one launch (y = r - T b and the z bits in registers, the
published column, junk rows, the parked timing-model factor and stage scratch in LDS /
global scratch).  If any of it leaked from one sweep into the next, a launch of S sweeps
would differ from S launches of one sweep each, where every sweep starts from fresh LDS and
registers.  So: one launch of S sweeps must equal S one-sweep launches BITWISE, records
and final state, for every build the host can pick (one chain per SIMD, two chains per
SIMD with the fair-priority counter, two waves per chain) -- VERDICT round 2, item 1.
"""
import numpy as np
import pytest

from gibbs_student_t_amd import _abi

from golden_io import load_ref
from test_gpu_parity import _native
from test_gpu_waves import KEYS, _init

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

FIXTURES = ("beta_efac_fixed", "c3_beta_fixed", "tm22_beta_fixed", "vvh17_prior")


def _ncu():
    return torch.cuda.get_device_properties(0).multi_processor_count


def _builds():
    # (label, chains, waves): wpb 1 / OCC 1 (C <= CUs), two waves per chain, and the
    # two-chains-per-SIMD build (C > 4 x CUs picks OCC = 2 and the progress counter)
    return (("occ1", 96, 1), ("pair", 96, 2), ("occ2", 4 * _ncu() + 64, 1))


@pytest.mark.parametrize("name", FIXTURES)
@pytest.mark.parametrize("build", ("occ1", "pair", "occ2"))
def test_one_launch_equals_single_sweep_launches(name, build):
    label, C, waves = next(b for b in _builds() if b[0] == build)
    ref = load_ref(name)
    S, seed, sweep0 = 100, 11, 5
    init = _init(ref, C, 21)

    ns = _native(ref, C, "persistent")
    ns.set_waves(waves)
    ns.set_state(**init)
    rec = ns.alloc_records(S)
    ns.sweep(S, records=rec, seed=seed, sweep0=sweep0)
    long_state = {k: v.clone() for k, v in ns.state.items()}
    ns.close()

    ns = _native(ref, C, "persistent")
    ns.set_waves(waves)
    ns.set_state(**init)
    bad = []
    for s in range(S):
        for k in KEYS:        # the state entering sweep s is record s of the long launch
            if not torch.equal(ns.state[k], rec[k][:, s]):
                bad.append((s, k))
        if bad:
            break
        ns.sweep(1, seed=seed, sweep0=sweep0 + s)
    if not bad:
        for k in KEYS + ("status",):
            if not torch.equal(ns.state[k], long_state[k]):
                bad.append((S, k))
    ns.close()
    assert not bad, f"{label}: first difference (sweep, array) {bad[:4]}"


@pytest.mark.parametrize("name", FIXTURES)
@pytest.mark.parametrize("build", ("occ1", "pair", "occ2"))
def test_poisoned_lds_and_scratch_change_nothing(name, build):
    """GST_DEBUG_POISON overwrites every chain's LDS (S0 / stage scratch, published columns,
    junk rows, MH variates, phi^-1) and its parked timing-model factor with NaN at the start
    of every sweep.  The chains must be bitwise those of an ordinary launch: no sweep reads
    a word it did not write itself (the stale-LDS hypothesis of VERDICT round 2, item 1)."""
    label, C, waves = next(b for b in _builds() if b[0] == build)
    ref = load_ref(name)
    S, seed, sweep0 = 100, 12, 9
    init = _init(ref, C, 22)
    outs = []
    for poison in (False, True):
        ns = _native(ref, C, "persistent")
        ns.set_waves(waves)
        ns.set_debug(poison=poison)
        ns.set_state(**init)
        rec = ns.alloc_records(S)
        ns.sweep(S, records=rec, seed=seed, sweep0=sweep0)
        outs.append(({k: v.clone() for k, v in rec.items()},
                     {k: v.clone() for k, v in ns.state.items()}))
        ns.close()
    (r0, s0), (r1, s1) = outs
    for k in KEYS:
        assert torch.equal(r0[k], r1[k]), f"{label}: record {k} differs under poisoning"
    for k in KEYS + ("status",):
        assert torch.equal(s0[k], s1[k]), f"{label}: final {k} differs under poisoning"
