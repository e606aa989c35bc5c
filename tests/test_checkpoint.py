"""Checkpoint format of the ``Gibbs`` sampler (sampler.make_checkpoint / check_checkpoint):
plain-array .npz round trip (no pickles) and the refusal of a checkpoint that does not fit
the sampler.  The bitwise resume itself runs on the GPU (test_gpu_sampler.py)."""
import numpy as np
import pytest

from gibbs_student_t_amd.sampler import check_checkpoint, dataset_fingerprint, make_checkpoint

CFG = dict(model="mixture", tdf=4, m=0.01, vary_df=True, theta_prior="beta",
           vary_alpha=True, alpha=1e10, pspin=None, exact_bdraw=False)


def _ck(C=3, n=7, m=5, P=3):
    rng = np.random.default_rng(0)
    return make_checkpoint(CFG, (n, m), 2**63 + 5, 1234, fingerprint="abc",
                           x=rng.normal(size=(C, P)), b=rng.normal(size=(C, m)),
                           z=rng.integers(0, 2, size=(C, n)).astype(float),
                           alpha=rng.uniform(1, 2, size=(C, n)), pout=rng.uniform(size=(C, n)),
                           theta=rng.uniform(size=C), nu=rng.integers(1, 31, size=C))


def test_round_trip_through_npz(tmp_path):
    ck = _ck()
    p = tmp_path / "ck.npz"
    np.savez(p, **ck)
    with np.load(p, allow_pickle=False) as f:
        back = {k: f[k] for k in f.files}
    assert set(back) == set(ck)
    for k in ck:
        np.testing.assert_array_equal(back[k], ck[k])
    assert int(back["seed"]) == 2**63 + 5 and int(back["sweep_counter"]) == 1234
    check_checkpoint(back, CFG, (7, 5), 3)


@pytest.mark.parametrize("change", ["model", "shape", "chains", "version", "dataset"])
def test_mismatch_is_refused(change):
    ck = _ck()
    cfg, shape, C = dict(CFG), (7, 5), 3
    if change == "model":
        cfg["model"] = "t"
    elif change == "shape":
        shape = (7, 6)
    elif change == "chains":
        C = 4
    elif change == "dataset":
        with pytest.raises(ValueError, match="different dataset"):
            check_checkpoint(ck, cfg, shape, C, fingerprint="abd")
        return
    else:
        ck["version"] = np.int64(99)
    with pytest.raises(ValueError):
        check_checkpoint(ck, cfg, shape, C)


def test_equal_option_values_are_accepted():
    """tdf = 4 vs 4.0, m = np.float64(0.01) vs 0.01: the same options."""
    ck = _ck()
    cfg = dict(CFG, tdf=4.0, m=np.float64(0.01), alpha=np.float64(1e10), vary_df=np.bool_(True))
    check_checkpoint(ck, cfg, (7, 5), 3, fingerprint="abc")


def test_fingerprint_tells_datasets_apart():
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from golden_io import load_dataset
    a, b = load_dataset(), load_dataset(dataset="c3")
    assert dataset_fingerprint(a) == dataset_fingerprint(load_dataset())
    assert dataset_fingerprint(a) != dataset_fingerprint(b)
    # same shape, one residual changed
    c = load_dataset()
    c._r = c._r.copy()
    c._r[3] += 1e-9
    assert dataset_fingerprint(c) != dataset_fingerprint(a)
