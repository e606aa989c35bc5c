"""Escape sweeps of vvh17 chains from the all-outlier start, by the REFERENCE itself.

    OPENBLAS_NUM_THREADS=1 python tools/vvh17_escape_reference.py [--seeds 256] [--seed0 20000]
        [--sweeps 1000] [--procs 8] [--golden tests/golden/vvh17_escape_ref.json]
        [--check-oracle N]

Imports /root/reference/gibbs.py (its only shim: Python-2 ``map``, as tools/gen_golden.py)
and runs ``Gibbs(pta, **run_sims.MODELS['vvh17']).sample(xs, niter)`` on the golden J1713
dataset from the prior draw ``np.random.seed(seed); xs = pta.sample_params()``
(run_sims.py:111), one chain per seed.  The reference starts vvh17 with z = 1 (gibbs.py:50-51)
and alpha = 1e10 (gibbs.py:44-45); a chain's escape sweep is the first i with
sum(zchain[i]) < n / 2 (zchain[i] = the state after i sweeps, gibbs.py:355-361), None if it
stays until ``--sweeps``.  Only the escape sweeps are written (tests/golden/, for
tests/test_gpu_ks.py); the reference never travels.

``--check-oracle N`` also replays the first N seeds with the oracle (gibbs.py's algorithm,
legacy MT19937, SVD draw; tools/vvh17_escape.py's ``svd`` variant) and asserts the same escape
sweeps, which pins that tool's floor-rule calibration runs to the reference.
"""
from __future__ import annotations

import argparse
import builtins
import json
import os
import sys
import time
import warnings
from multiprocessing import Pool

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def ref_escape(args):
    seed, sweeps = args
    sys.dont_write_bytecode = True
    if "/root/reference" not in sys.path:
        sys.path.insert(0, "/root/reference")
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import gibbs as refgibbs  # the reference
    from golden_io import load_dataset
    from gibbs_student_t_amd.run_sims import MODELS
    refgibbs.map = lambda f, *a: list(builtins.map(f, *a))
    warnings.filterwarnings("ignore")
    pta = load_dataset()
    np.random.seed(seed)
    xs = pta.sample_params()
    g = refgibbs.Gibbs(pta, **MODELS["vvh17"])
    sys.stdout = open(os.devnull, "w")        # gibbs.py:382-385's progress line
    n = len(pta.get_residuals()[0])
    # one sample() call: gibbs.py keeps the parameter vector after a sweep only in
    # sample()'s local ``xnew``, so a run cannot be continued in pieces
    g.sample(xs, niter=sweeps + 1)
    hit = np.flatnonzero(g.zchain.sum(axis=1)[1:] < n / 2)
    return seed, (int(hit[0]) + 1 if hit.size else None)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, default=256)
    ap.add_argument("--seed0", type=int, default=20000)
    ap.add_argument("--sweeps", type=int, default=1000)
    ap.add_argument("--procs", type=int, default=8)
    ap.add_argument("--golden", default=None)
    ap.add_argument("--check-oracle", type=int, default=0)
    a = ap.parse_args()
    t0 = time.time()
    with Pool(a.procs) as pool:
        res = pool.map(ref_escape, [(a.seed0 + s, a.sweeps) for s in range(a.seeds)],
                       chunksize=1)
    esc = [e for _, e in sorted(res)]
    e = np.array([v if v is not None else a.sweeps + 1 for v in esc])
    print(f"reference: {a.seeds} chains, median escape {np.median(e)}, trapped at 200/500: "
          f"{np.mean(e > 200):.3f}/{np.mean(e > 500):.3f}, {time.time() - t0:.0f} s", flush=True)
    if a.check_oracle:
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import vvh17_escape as ve
        with Pool(a.procs) as pool:
            orc = pool.map(ve.run_one, [("svd", a.seed0 + s, a.sweeps, "j1713")
                                        for s in range(a.check_oracle)], chunksize=1)
        oe = [r[2] for r in sorted(orc, key=lambda r: r[1])]
        bad = [(a.seed0 + i, x, y) for i, (x, y) in enumerate(zip(esc[:a.check_oracle], oe))
               if x != y]
        print(f"oracle svd variant vs reference on {a.check_oracle} seeds: "
              f"{len(bad)} differ {bad[:5]}")
        assert not bad
    if a.golden:
        g = {"source": "tools/vvh17_escape_reference.py: /root/reference/gibbs.py imported "
                       "(map shim only), Gibbs(model='vvh17', run_sims kwargs).sample from "
                       "prior draws np.random.seed(seed)",
             "dataset": "j1713", "seeds": a.seeds, "seed0": a.seed0, "sweeps": a.sweeps,
             "criterion": "first sweep with sum z < n/2", "escape": esc}
        with open(a.golden, "w") as f:
            json.dump(g, f)


if __name__ == "__main__":
    main()
