"""CPU study: escape of vvh17 chains from the reference's all-outlier start, per b-draw rule.

    OPENBLAS_NUM_THREADS=1 python tools/vvh17_escape.py [--seeds 48] [--sweeps 1500]
        [--variants svd,exact,floor0.5] [--dataset j1713|c4:IDX] [--out FILE.json]

The reference starts vvh17 chains with every TOA flagged (z = 1, gibbs.py:50-51) and alpha
fixed at 1e10 (gibbs.py:44-45).  Sigma then has cond ~ 1e22, and the reference's SVD
(gibbs.py:169-171) returns the smallest eigenvalues at LAPACK's rounding floor, which
narrows the timing-model part of the b draw until some TOAs fit again and the chain leaves
the state.  Each variant runs the oracle (bit-exact to gibbs.py with the legacy RNG) from
the same prior draws with one b-draw rule:

* ``svd``: the reference's own draw (u (u^T d / s) + u s^-1/2 xi);
* ``exact``: the exact Cholesky draw from Sigma;
* ``floorC`` / ``floorC@G``: the HIP path's rule (oracle ``Oracle.floor_shift``): exact draw
  from Sigma + f I with f = C x 2^-52 x the largest pivot when the smallest pivot is below G x
  2^-52 of it (G defaults to the oracle's FLOOR_GATE).

The ``svd`` variant reproduces the reference's own escape sweeps exactly (checked against
/root/reference/gibbs.py itself by tools/vvh17_escape_reference.py --check-oracle).

Prints and writes the escape sweep (first sweep whose z has sum < n / 2) per seed, the
trapped fraction at sweeps 100 / 200 / 500 / 1000, and a two-sample KS test of each
variant's escape times against ``svd``'s (censored at --sweeps).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
import warnings
from multiprocessing import Pool

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def _setup(dataset):
    from gibbs_student_t_amd.run_sims import MODELS
    from oracle.gibbs_oracle import OutlierModel
    if dataset == "j1713":
        from golden_io import load_dataset
        pta = load_dataset()
    else:                       # c4:IDX -> config-4 dataset IDX (bench.workload order)
        import bench
        from gibbs_student_t_amd import run_sims
        idx = int(dataset.split(":")[1])
        grid = run_sims.build_grid(thetas=(0.05, 0.1, 0.15), realisations=5,
                                   dofs=(None, 4.0))[:bench.CONFIG4_DATASETS]
        pta = grid[idx].pta
    return pta, OutlierModel(**MODELS["vvh17"])


import oracle.gibbs_oracle as _go  # noqa: E402

GATE0, C0 = _go.FLOOR_GATE, _go.FLOOR_C


def run_one(args):
    variant, seed, sweeps, dataset = args
    warnings.simplefilter("ignore")
    import oracle.gibbs_oracle as go
    pta, cfg = _setup(dataset)
    orc = go.Oracle(pta, cfg)
    mean = "svd"
    go.FLOOR_GATE, go.FLOOR_C = GATE0, C0     # pool workers are reused: reset every job
    if variant == "exact":
        go.FLOOR_GATE = 0.0
        mean = "floor"
    elif variant.startswith("floor"):
        # floorC or floorC@G: f = C x 2^-52 x the largest pivot, gate G x 2^-52
        c, _, g = variant[5:].partition("@")
        go.FLOOR_C = float(c)
        if g:
            go.FLOOR_GATE = float(g) * 2.0 ** -52
        mean = "floor"
    np.random.seed(seed)
    x = pta.sample_params()
    st = go.initial_state(pta, cfg)
    src = go.LegacyNumpyVariates()
    n = orc.n
    esc = None
    sz = []
    for i in range(sweeps):
        x = orc.sweep(st, x, src, b_mean=mean)
        s = int(np.sum(st.z))
        if i % 50 == 49:
            sz.append(s)
        if esc is None and s < n / 2:
            esc = i + 1
            if variant != "svd" or i >= 200:
                break
    return variant, seed, esc, sz


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, default=48)
    ap.add_argument("--seed0", type=int, default=5000)
    ap.add_argument("--sweeps", type=int, default=1500)
    ap.add_argument("--variants", default="svd,exact,floor0.25,floor0.5,floor1")
    ap.add_argument("--dataset", default="j1713")
    ap.add_argument("--procs", type=int, default=8)
    ap.add_argument("--out", default=None)
    ap.add_argument("--golden", default=None,
                    help="also write the svd (reference) variant's escape sweeps here "
                         "(tests/golden/vvh17_escape_ref.json)")
    ap.add_argument("--ref-json", default=None,
                    help="take the svd variant's escape sweeps from this reference file "
                         "(tools/vvh17_escape_reference.py --golden) instead of running it")
    ap.add_argument("--golden-from", default=None,
                    help="only write --golden from an earlier --out file")
    a = ap.parse_args()
    if a.golden_from:
        with open(a.golden_from) as f:
            write_golden(json.load(f), a.golden)
        return
    variants = a.variants.split(",")
    refrows = []
    if a.ref_json:
        with open(a.ref_json) as f:
            rj = json.load(f)
        assert rj["seed0"] == a.seed0 and rj["seeds"] >= a.seeds and rj["sweeps"] == a.sweeps
        refrows = [("svd", a.seed0 + i, e, []) for i, e in enumerate(rj["escape"][:a.seeds])]
        variants = ["svd"] + [v for v in variants if v != "svd"]
    jobs = [(v, a.seed0 + s, a.sweeps, a.dataset) for v in variants for s in range(a.seeds)
            if not (a.ref_json and v == "svd")]
    t0 = time.time()
    with Pool(a.procs) as pool:
        res = refrows + pool.map(run_one, jobs, chunksize=1)
    from scipy.stats import ks_2samp
    out = {"dataset": a.dataset, "seeds": a.seeds, "seed0": a.seed0, "sweeps": a.sweeps,
           "criterion": "first sweep with sum z < n/2", "variants": {}}
    by = {v: [r for r in res if r[0] == v] for v in variants}
    cens = lambda v: np.array([r[2] if r[2] is not None else a.sweeps + 1 for r in by[v]])
    for v in variants:
        e = cens(v)
        row = {"escape": [int(x) if x <= a.sweeps else None for x in e],
               "median": float(np.median(e)),
               "trapped_frac": {str(k): float(np.mean(e > k)) for k in (50, 100, 200, 500, 1000)
                                if k <= a.sweeps}}
        if v != "svd" and "svd" in by:
            ks = ks_2samp(e, cens("svd"))
            row["ks_vs_svd"] = {"stat": float(ks.statistic), "p": float(ks.pvalue)}
        out["variants"][v] = row
        print(f"{v:10s} median {row['median']:7.1f}  trapped {row['trapped_frac']}  "
              f"{row.get('ks_vs_svd', '')}", flush=True)
    out["cpu_seconds_wall"] = time.time() - t0
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)
    if a.golden:
        write_golden(out, a.golden)


def write_golden(out, path):
    """The reference algorithm's escape sweeps (svd variant: the oracle, bit-exact to gibbs.py
    with its legacy RNG and SVD draw) for tests/test_gpu_ks.py."""
    g = {"source": "tools/vvh17_escape.py svd variant (oracle = gibbs.py algorithm, legacy "
                   "MT19937, SVD b draw)", "dataset": out["dataset"], "seeds": out["seeds"],
         "seed0": out["seed0"], "sweeps": out["sweeps"], "criterion": out["criterion"],
         "escape": out["variants"]["svd"]["escape"]}
    with open(path, "w") as f:
        json.dump(g, f)


if __name__ == "__main__":
    main()
