"""BASELINE config 4 at its full size on one GPU: the run_sims.py grid of 256 simulated
datasets x 64 chains = 16384 chains in one ragged batch.

Property checks (no oracle at this size): every chain's status is clean, every state value
is finite, x stays in its prior box (gibbs.py:337-339 rejects everything outside), theta in
[0, 1], nu in 1..30, z in {0, 1}, alpha > 0; and the batch equals a 2-shard split of the
same datasets bitwise (the multi-GPU partition of bench.py --config 4: datasets sharded,
Philox keyed by global chain id)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a HIP device", allow_module_level=True)

import bench  # noqa: E402
from gibbs_student_t_amd._abi import STATUS_ERRORS, STATUS_FLOOR  # noqa: E402
from gibbs_student_t_amd.native import NativeSampler  # noqa: E402

S, SEED = 40, 404


def _run(rank, world):
    wl = bench.workload(4, rank, world, None)
    ns = NativeSampler(wl["ptas"], wl["cfgs"], 0)
    ns.alloc(wl["C"], dataset=wl["ds"])
    ns.set_state(**wl["init"])
    ns.sweep(S, seed=SEED, sweep0=0, chain0=wl["chain0"])
    out = ns.get_state()
    ns.close()
    return wl, out


def test_config4_full_grid_properties_and_shard_split():
    wl, full = _run(0, 1)
    assert wl["C"] == 256 * 64
    assert np.all((full["status"] & STATUS_ERRORS) == 0)
    for k in ("x", "b", "z", "alpha", "pout", "theta", "nu"):
        assert np.all(np.isfinite(full[k])), k
    for d, (pta, cfg) in enumerate(zip(wl["ptas"], wl["cfgs"])):
        sel = wl["ds"] == d
        lo = np.array([p.pmin for p in pta.params])
        hi = np.array([p.pmax for p in pta.params])
        x = full["x"][sel]
        assert np.all((x >= lo) & (x <= hi)), d
        z = full["z"][sel][:, :pta.n]
        assert np.all((z == 0) | (z == 1)), d
        assert np.all(full["alpha"][sel][:, :pta.n] > 0), d
    assert np.all((full["theta"] >= 0) & (full["theta"] <= 1))
    assert np.all((full["nu"] >= 1) & (full["nu"] <= 30) & (full["nu"] == np.round(full["nu"])))
    # two shards of 128 datasets each (bench.py --gpus 2 --config 4) == the single batch
    parts = [_run(r, 2) for r in range(2)]
    C2 = parts[0][0]["C"]
    assert C2 * 2 == wl["C"]
    for r, (wlr, out) in enumerate(parts):
        rows = slice(r * C2, (r + 1) * C2)
        nst = out["z"].shape[1]
        for k in ("x", "b", "theta", "nu", "status"):
            np.testing.assert_array_equal(out[k], full[k][rows], err_msg=f"shard {r} {k}")
        for k in ("z", "alpha", "pout"):
            np.testing.assert_array_equal(out[k], full[k][rows][:, :nst],
                                          err_msg=f"shard {r} {k}")
