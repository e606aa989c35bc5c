"""Dataset batches on the GPU: many (dataset, outlier model) pairs in one launch.

run_sims.py:80-113 runs every simulated pulsar (outlier / no_outlier twin of
simulate_data.py, whose n differ) under five outlier models.  The sampler batches such a
grid into one launch: each chain names its dataset (gst_state.dataset), per-TOA arrays use
the batch's largest n as row stride.  Parity: every chain of a batch must reproduce its own
reference fixture (same tolerances as test_gpu_parity.py) and, in Philox mode, be bitwise
identical to a launch of its dataset alone.
"""
import numpy as np
import pytest

from golden_io import fixture_names, load_ref, oracle_replay, sweep_state

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a HIP device", allow_module_level=True)

from gibbs_student_t_amd._abi import STATUS_ERRORS, STATUS_FLOOR  # noqa: E402
from gibbs_student_t_amd.native import NativeSampler, pack_tape  # noqa: E402
from test_gpu_parity import assert_replay_matches  # noqa: E402

# three-parameter fixtures the single-chain replay covers (test_full_chain_replay), plus the
# ragged no_outlier twin (n = 119 next to n = 130)
REPLAY = [n for n in fixture_names()
          if "fixed" in n and "vvh17" not in n and "efac" not in n
          and not n.startswith(("scaled", "c20", "tm22", "mb", "ec", "ebig", "jb"))]   # one basis shape per batch


def _pad(a, nst):
    out = np.zeros(a.shape[:-1] + (nst,))
    out[..., :a.shape[-1]] = a
    return out


def test_batch_replays_every_fixture():
    assert any(n.startswith("simclean") for n in REPLAY)
    refs = [load_ref(n) for n in REPLAY]
    ns = NativeSampler([r["pta"] for r in refs], [r["kw"] for r in refs], 0)
    C = len(refs)
    ns.alloc(C, dataset=np.arange(C))
    nst = ns.n
    assert nst == max(r["pta"].n for r in refs) and min(r["pta"].n for r in refs) < nst
    S = int(refs[0]["niter"])
    s0 = [sweep_state(r, 0) for r in refs]
    ns.set_state(x=np.stack([r["xs"] for r in refs]), b=np.stack([s["b"] for s in s0]),
                 z=np.stack([_pad(s["z"], nst) for s in s0]),
                 alpha=np.stack([_pad(s["alpha"], nst) for s in s0]),
                 pout=np.stack([_pad(s["pout"], nst) for s in s0]),
                 theta=np.array([s["theta"] for s in s0]), nu=np.array([s["nu"] for s in s0]))
    tape = np.stack([pack_tape(r["tape"], np.arange(S), r["pta"].n, ns.m, ns.stride, nst)
                     for r in refs])
    rec = ns.alloc_records(S)
    for v in rec.values():
        v.zero_()
    ns.sweep(S, records=rec, tape=torch.as_tensor(tape).to(ns.tdev).contiguous())
    got = {k: v.cpu().numpy() for k, v in rec.items()}
    assert np.all((ns.get_state()["status"] & STATUS_ERRORS) == 0)
    for c, (name, r) in enumerate(zip(REPLAY, refs)):
        n = r["pta"].n
        # 1e-10 against the oracle's Cholesky-mean replay of the same tape ...
        assert_replay_matches({k: v[c] for k, v in got.items()}, oracle_replay(r, S), r,
                              name)
        # ... and the reference's own (SVD-mean) chain, whose mean error compounds
        np.testing.assert_array_equal(got["x"][c], r["chain"], err_msg=name)
        np.testing.assert_array_equal(got["z"][c][:, :n], r["zchain"], err_msg=name)
        np.testing.assert_array_equal(got["nu"][c], r["dfchain"], err_msg=name)
        for k, rk in (("b", "bchain"), ("alpha", "alphachain"), ("pout", "poutchain"),
                      ("theta", "thetachain")):
            g = got[k][c][..., :n] if k in ("alpha", "pout") else got[k][c]
            rel = np.abs(g - r[rk]) / np.maximum(np.abs(r[rk]), 1e-300)
            assert np.all(rel <= 1e-6), f"{name} {k}: max rel {rel.max():.3e}"
        # TOAs beyond this dataset's n are never written
        assert np.all(got["alpha"][c][:, n:] == 0.0) if n < nst else True


def test_batch_equals_single_dataset_launches():
    """Philox mode: chains in a ragged multi-model batch == their dataset launched alone."""
    names = ["beta_fixed", "simclean_beta_fixed", "sim_t_fixed", "simclean_vvh17_fixed"]
    refs = [load_ref(n) for n in names]
    per, S, seed = 6, 7, 4242
    C = per * len(refs)
    ds = np.repeat(np.arange(len(refs)), per)
    big = NativeSampler([r["pta"] for r in refs], [r["kw"] for r in refs], 0)
    big.alloc(C, dataset=ds)
    nst = big.n

    def init(r, k, width):
        s = sweep_state(r, 0)
        return dict(x=np.tile(r["xs"], (k, 1)), b=np.tile(s["b"], (k, 1)),
                    z=np.tile(_pad(s["z"], width), (k, 1)),
                    alpha=np.tile(_pad(s["alpha"], width), (k, 1)),
                    pout=np.tile(_pad(s["pout"], width), (k, 1)),
                    theta=np.full(k, s["theta"]), nu=np.full(k, s["nu"]))

    parts = [init(r, per, nst) for r in refs]
    big.set_state(**{k: np.concatenate([p[k] for p in parts]) for k in parts[0]})
    big.sweep(S, seed=seed, sweep0=3)
    full = big.get_state()
    assert np.all((full["status"] & STATUS_ERRORS) == 0)
    for d, r in enumerate(refs):
        one = NativeSampler(r["pta"], r["kw"], 0)
        one.alloc(per)
        one.set_state(**init(r, per, r["pta"].n))
        one.sweep(S, seed=seed, sweep0=3, chain0=d * per)
        o = one.get_state()
        sl = slice(d * per, (d + 1) * per)
        n = r["pta"].n
        for k in ("x", "b", "theta", "nu"):
            np.testing.assert_array_equal(full[k][sl], o[k], err_msg=f"{names[d]} {k}")
        for k in ("z", "alpha", "pout"):
            np.testing.assert_array_equal(full[k][sl][:, :n], o[k], err_msg=f"{names[d]} {k}")
        one.close()
    big.close()


def test_bad_dataset_index_is_flagged():
    r = load_ref("beta_fixed")
    ns = NativeSampler([r["pta"], r["pta"]], [r["kw"], r["kw"]], 0)
    with pytest.raises(ValueError):
        ns.alloc(2, dataset=[0, 2])
    ns.alloc(2, dataset=[0, 1])
    s = sweep_state(r, 0)
    ns.set_state(x=np.tile(r["xs"], (2, 1)), z=np.tile(s["z"], (2, 1)),
                 alpha=np.tile(s["alpha"], (2, 1)), theta=np.full(2, 0.01), nu=np.full(2, 4.0))
    ns.dataset.copy_(torch.tensor([0, 7], dtype=torch.int32, device=ns.tdev))
    ns.sweep(2, seed=1)
    st = ns.get_state()
    assert st["status"][0] == 0 and st["status"][1] == 4
    np.testing.assert_array_equal(st["x"][1], r["xs"])   # untouched
    ns.close()


def test_large_path_dataset_batch_equals_single_launches():
    """The large-model path batches datasets too (ragged n, 16-chain groups per dataset):
    each chain of a 2-dataset batch is bitwise its dataset's standalone launch."""
    from gibbs_student_t_amd import data
    from gibbs_student_t_amd.model import PTA
    from gibbs_student_t_amd.run_sims import MODELS
    ptas = [PTA(data.scaled_synthetic(n=n, components=40, ntm=100, seed=sd), components=40)
            for n, sd in ((1500, 11), (1333, 12))]
    cfgs = [MODELS["beta"], MODELS["t"]]
    per, S, seed = 16, 4, 99
    big = NativeSampler(ptas, cfgs, 0, path="large")
    assert big.path == "large"
    with pytest.raises(ValueError):
        big.alloc(2 * per, dataset=np.tile([0, 1], per))       # groups must not mix
    big.alloc(2 * per, dataset=np.repeat([0, 1], per))
    nst = big.n

    def init(pta, c0, width):
        lo = np.array([p.pmin for p in pta.params])
        hi = np.array([p.pmax for p in pta.params])
        x = np.stack([np.random.default_rng([3, c0 + c]).uniform(lo, hi) for c in range(per)])
        z = np.zeros((per, width))
        z[:, :pta.n] = 1.0
        return dict(x=x, b=np.zeros((per, pta.T.shape[1])), z=z, alpha=np.ones((per, width)),
                    pout=np.zeros((per, width)), theta=np.full(per, 0.01), nu=np.full(per, 4.0))

    parts = [init(p_, d * per, nst) for d, p_ in enumerate(ptas)]
    big.set_state(**{k: np.concatenate([p[k] for p in parts]) for k in parts[0]})
    big.sweep(S, seed=seed, sweep0=1)
    full = big.get_state()
    assert np.all((full["status"] & STATUS_ERRORS) == 0)
    for d, (p_, cfg) in enumerate(zip(ptas, cfgs)):
        one = NativeSampler(p_, cfg, 0, path="large")
        one.alloc(per)
        one.set_state(**init(p_, d * per, p_.n))
        one.sweep(S, seed=seed, sweep0=1, chain0=d * per)
        o = one.get_state()
        sl = slice(d * per, (d + 1) * per)
        for k in ("x", "b", "theta", "nu"):
            np.testing.assert_array_equal(full[k][sl], o[k], err_msg=f"dataset {d} {k}")
        for k in ("z", "alpha", "pout"):
            np.testing.assert_array_equal(full[k][sl][:, :p_.n], o[k], err_msg=f"dataset {d} {k}")
        one.close()
    big.close()


def test_large_path_chains_do_not_depend_on_batch_partners():
    """A dataset's chains on the large path are bitwise the same launched alone or batched
    with datasets of other kernel classes: n <= 8k (one-wave white pass), 8k < n <= 32k (256
    threads) and n > 32k TOAs (1024 threads), per-TOA block sizes and hyper kernels being
    chosen per dataset, not from the batch (run_sims.py:80-113 runs each
    dataset as an independent Gibbs object)."""
    from gibbs_student_t_amd import data
    from gibbs_student_t_amd.model import PTA
    from gibbs_student_t_amd.run_sims import MODELS
    ptas = [PTA(data.scaled_synthetic(n=n, components=30, ntm=14, seed=sd), components=30)
            for n, sd in ((1000, 21), (9000, 22), (33000, 23))]
    cfg = MODELS["beta"]
    per, S, seed = 16, 3, 5

    def init(pta, c0, width):
        lo = np.array([p.pmin for p in pta.params])
        hi = np.array([p.pmax for p in pta.params])
        x = np.stack([np.random.default_rng([7, c0 + c]).uniform(lo, hi) for c in range(per)])
        z = np.zeros((per, width))
        z[:, :pta.n] = 1.0
        return dict(x=x, b=np.zeros((per, pta.T.shape[1])), z=z, alpha=np.ones((per, width)),
                    pout=np.zeros((per, width)), theta=np.full(per, 0.01), nu=np.full(per, 4.0))

    def alone(d, j):
        one = NativeSampler(ptas[d], cfg, 0, path="large")
        one.alloc(per)
        one.set_state(**init(ptas[d], j * per, ptas[d].n))
        one.sweep(S, seed=seed, sweep0=2, chain0=j * per)   # the chains' global ids
        out = one.get_state()
        one.close()
        return out

    for members in ((0, 1), (2, 0), (1, 2), (0, 1, 2)):
        big = NativeSampler([ptas[d] for d in members], [cfg] * len(members), 0, path="large")
        big.alloc(len(members) * per, dataset=np.repeat(np.arange(len(members)), per))
        nst = big.n
        parts = [init(ptas[d], j * per, nst) for j, d in enumerate(members)]
        big.set_state(**{k: np.concatenate([p[k] for p in parts]) for k in parts[0]})
        big.sweep(S, seed=seed, sweep0=2)
        full = big.get_state()
        big.close()
        assert np.all((full["status"] & STATUS_ERRORS) == 0)
        for j, d in enumerate(members):
            ref = alone(d, j)
            sl = slice(j * per, (j + 1) * per)
            n = ptas[d].n
            for k in ("x", "b", "theta", "nu"):
                np.testing.assert_array_equal(full[k][sl], ref[k], err_msg=f"{members} {d} {k}")
            for k in ("z", "alpha", "pout"):
                np.testing.assert_array_equal(full[k][sl][:, :n], ref[k][:, :n],
                                              err_msg=f"{members} {d} {k}")


def test_general_white_noise_batch_matches_single_datasets():
    """The persistent kernel's general white-noise instances (per-backend efac / equad, ECORR;
    DESIGN.md 4d) in a batch of two structurally equal datasets -- ``ecb`` (every TOA its own
    error bar: per-TOA likelihood, MFMA Gram) and ``ecq`` (four noise classes: class
    likelihood, low-rank Gram) -- give each dataset's chains bitwise as when it runs alone:
    every per-dataset table (TOA backends, ECORR column backends, noise classes and their
    backends, class Grams) is read from the chain's own dataset."""
    refs = [load_ref("ecb_beta_fixed"), load_ref("ecq_beta_fixed")]
    per, S, seed = 24, 6, 9

    def init(ref, c0):
        pta = ref["pta"]
        lo = np.array([p.pmin for p in pta.params])
        hi = np.array([p.pmax for p in pta.params])
        s0 = sweep_state(ref, 0)
        return dict(x=np.stack([np.random.default_rng([11, c0 + c]).uniform(lo, hi)
                                for c in range(per)]),
                    b=np.tile(s0["b"], (per, 1)), z=np.tile(s0["z"], (per, 1)),
                    alpha=np.tile(s0["alpha"], (per, 1)), pout=np.tile(s0["pout"], (per, 1)),
                    theta=np.full(per, s0["theta"]), nu=np.full(per, s0["nu"]))

    big = NativeSampler([r["pta"] for r in refs], [r["kw"] for r in refs], 0, path="persistent")
    big.alloc(2 * per, dataset=np.repeat(np.arange(2), per))
    parts = [init(r, j * per) for j, r in enumerate(refs)]
    big.set_state(**{k: np.concatenate([p[k] for p in parts]) for k in parts[0]})
    big.sweep(S, seed=seed, sweep0=3)
    full = big.get_state()
    big.close()
    assert np.all((full["status"] & STATUS_ERRORS) == 0)
    for j, ref in enumerate(refs):
        one = NativeSampler(ref["pta"], ref["kw"], 0, path="persistent")
        one.alloc(per)
        one.set_state(**parts[j])
        one.sweep(S, seed=seed, sweep0=3, chain0=j * per)
        alone = one.get_state()
        one.close()
        sl = slice(j * per, (j + 1) * per)
        for k in ("x", "b", "z", "alpha", "pout", "theta", "nu", "status"):
            np.testing.assert_array_equal(full[k][sl], alone[k], err_msg=f"dataset {j} {k}")
