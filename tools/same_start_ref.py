"""Same-start reference trajectories for the ECORR-heavy posteriors.

The long-run KS layer needs a converged reference, and on ``mb`` (20 Fourier + 60 ECORR
columns, two backends) the reference's own 8 x 25000-sweep chains disagree with one another
(DESIGN.md 4d).  A test that needs no convergence: chains started from the SAME initial states
and run through the same transition kernel have the same law at every sweep, so the GPU's
chains at sweep s and the reference's chains at sweep s -- one per start, independent across
starts -- must pass two-sample tests whatever the mixing.  This runs the REFERENCE itself
(/root/reference/gibbs.py, imported with its only shim, the Python-2 ``map``) from C prior
draws (``np.random.default_rng([SEED, c])``) and gibbs.py:29-51's latent start, S sweeps
each, and keeps every THIN-th record of x, theta and nu (``Gibbs.sample`` records the state
at the start of each sweep, gibbs.py:355-361).  Only the ``.npz`` of draws is committed
(tests/golden/samestart_<dataset>_<model>.npz); tests/test_gpu_ks.py runs the GPU chains
from the same starts.

    python tools/same_start_ref.py DATASET MODEL CHAINS SWEEPS [THIN] [NPROC]
"""
from __future__ import annotations

import builtins
import os
import subprocess
import sys
import time
import warnings

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
OUT = os.path.join(ROOT, "tests", "golden")
SEED = 424242


def start(pta, c):
    lo = np.array([p.pmin for p in pta.params])
    hi = np.array([p.pmax for p in pta.params])
    return np.random.default_rng([SEED, c]).uniform(lo, hi)


def worker(dataset, model, c0, c1, sweeps, thin, path):
    sys.dont_write_bytecode = True
    sys.path.insert(0, "/root/reference")
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import gibbs as refgibbs  # the reference
    from golden_io import load_dataset
    from gibbs_student_t_amd.run_sims import MODELS
    refgibbs.map = lambda f, *a: list(builtins.map(f, *a))
    warnings.filterwarnings("ignore")
    pta = load_dataset(dataset=dataset)
    xs, th, nu = [], [], []
    for c in range(c0, c1):
        np.random.seed(SEED + c)
        g = refgibbs.Gibbs(pta, **MODELS[model])
        g.sample(start(pta, c), niter=sweeps)
        xs.append(g.chain[::thin])
        th.append(g.thetachain[::thin])
        nu.append(g.dfchain[::thin])
    np.savez(path, x=np.array(xs), theta=np.array(th), nu=np.array(nu))


def main():
    if sys.argv[1:2] == ["--worker"]:
        a = sys.argv[2:]
        worker(a[0], a[1], int(a[2]), int(a[3]), int(a[4]), int(a[5]), a[6])
        return
    dataset, model = sys.argv[1], sys.argv[2]
    chains, sweeps = int(sys.argv[3]), int(sys.argv[4])
    thin = int(sys.argv[5]) if len(sys.argv) > 5 else 10
    nproc = int(sys.argv[6]) if len(sys.argv) > 6 else 8
    env = dict(os.environ, OPENBLAS_NUM_THREADS="1", OMP_NUM_THREADS="1", MKL_NUM_THREADS="1")
    bounds = np.linspace(0, chains, nproc + 1).astype(int)
    tmp = [f"/tmp/gst_samestart_{dataset}_{model}_{k}.npz" for k in range(nproc)]
    t0 = time.time()
    procs = [subprocess.Popen([sys.executable, __file__, "--worker", dataset, model,
                               str(bounds[k]), str(bounds[k + 1]), str(sweeps), str(thin),
                               tmp[k]], env=env) for k in range(nproc)]
    for p in procs:
        assert p.wait() == 0
    parts = [np.load(t) for t in tmp]
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from golden_io import load_dataset
    pta = load_dataset(dataset=dataset)
    out = dict(x=np.concatenate([p["x"] for p in parts]),
               theta=np.concatenate([p["theta"] for p in parts]),
               nu=np.concatenate([p["nu"] for p in parts]),
               x0=np.stack([start(pta, c) for c in range(chains)]),
               names=np.array(pta.param_names), seed=SEED, sweeps=sweeps, thin=thin,
               model=model, dataset=dataset, secs=time.time() - t0)
    np.savez_compressed(os.path.join(OUT, f"samestart_{dataset}_{model}.npz"), **out)
    for t in tmp:
        os.remove(t)
    print({k: v.shape for k, v in out.items() if hasattr(v, "shape")}, f"{time.time() - t0:.0f} s")


if __name__ == "__main__":
    main()
