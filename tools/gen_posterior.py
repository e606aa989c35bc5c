"""Reference posterior samples for the KS layer of the parity contract (north star).

Runs the REFERENCE sampler (/root/reference/gibbs.py, only shim: Python-2 ``map``) in
this container on the golden J1713+0747 dataset (tests/golden/j1713_dataset.npz), one
chain per process with single-threaded BLAS, from prior draws (run_sims.py:111), and
keeps thinned post-burn-in draws of the sampled parameters, theta and nu.  Only the
``.npz`` of draws is committed (tests/golden/posterior_ref_*.npz); tests/test_gpu_ks.py
compares the GPU chains' marginals with them by two-sample KS tests.

    python tools/gen_posterior.py [model] [sweeps_per_chain] [chains] [dataset]

``dataset`` (default j1713): a golden dataset name, e.g. ``ecb`` / ``ecq`` (per-backend efac /
equad and ECORR: the persistent kernel's general white-noise instances) -> posterior_ref_<dataset>_<model>.npz.
"""
from __future__ import annotations

import builtins
import os
import subprocess
import sys
import warnings

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
OUT = os.path.join(ROOT, "tests", "golden")
BURN, THIN = 1000, 25


def worker(model, sweeps, seed, path, dataset="j1713"):
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
    np.random.seed(seed)
    xs = pta.sample_params()
    g = refgibbs.Gibbs(pta, **MODELS[model])
    g.sample(xs, niter=sweeps)
    sl = slice(BURN, None, THIN)
    np.savez(path, x=g.chain[sl], theta=g.thetachain[sl], nu=g.dfchain[sl],
             names=np.array(pta.param_names))


def main():
    if sys.argv[1:2] == ["--worker"]:
        worker(sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), sys.argv[5], sys.argv[6])
        return
    model = sys.argv[1] if len(sys.argv) > 1 else "beta"
    sweeps = int(sys.argv[2]) if len(sys.argv) > 2 else 25000
    chains = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    dataset = sys.argv[4] if len(sys.argv) > 4 else "j1713"
    env = dict(os.environ, OPENBLAS_NUM_THREADS="1", OMP_NUM_THREADS="1", MKL_NUM_THREADS="1")
    tmp = [f"/tmp/gst_post_{dataset}_{model}_{c}.npz" for c in range(chains)]
    procs = [subprocess.Popen([sys.executable, __file__, "--worker", model, str(sweeps),
                               str(9000 + c), tmp[c], dataset], env=env) for c in range(chains)]
    for p in procs:
        assert p.wait() == 0
    parts = [np.load(t) for t in tmp]
    out = dict(x=np.stack([p["x"] for p in parts]), theta=np.stack([p["theta"] for p in parts]),
               nu=np.stack([p["nu"] for p in parts]), names=parts[0]["names"],
               burn=BURN, thin=THIN, sweeps=sweeps, model=model)
    np.savez_compressed(os.path.join(OUT, f"posterior_ref_{dataset}_{model}.npz"), **out)
    for t in tmp:
        os.remove(t)
    print({k: v.shape for k, v in out.items() if hasattr(v, "shape")})


if __name__ == "__main__":
    main()
