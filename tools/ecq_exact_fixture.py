"""tests/golden/posterior_exact_ecq_beta.npz from tools/ecq_theta_bias.py's ``numpy-floor`` run.

That run is the reference algorithm -- the oracle making gibbs.py's own legacy RNG calls,
its samplers, stage order and MH -- with ONE change: b drawn exactly (Cholesky; the SVD noise
floor rule only where Sigma is beyond fp64 resolution, Oracle.floor_shift), where gibbs.py
maps normals through sl.svd(Sigma) (gibbs.py:169-180).  16 chains x 50000 sweeps from prior
draws (seeds 31000 + c), burn-in 1000; this keeps every 25th sweep (the layout of
posterior_ref_*.npz, tools/gen_posterior.py).  tests/test_gpu_ks.py compares the GPU's ecq
posterior with it (the reference's SVD draw moves theta by ~1%).

    python tools/ecq_theta_bias.py 50000 16 ecq numpy-floor   (writes /tmp/gst_theta_bias/)
    python tools/ecq_exact_fixture.py
"""
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    from golden_io import load_dataset
    d = np.load("/tmp/gst_theta_bias/ecq_numpy-floor_all.npz")
    k = 5                       # the run kept every 5th sweep; keep every 25th
    pta = load_dataset(dataset="ecq")
    np.savez_compressed(os.path.join(ROOT, "tests", "golden", "posterior_exact_ecq_beta.npz"),
                        x=d["x"][:, ::k], theta=d["theta"][:, ::k], nu=d["nu"][:, ::k],
                        names=np.array(pta.param_names), burn=1000, thin=25, sweeps=50000,
                        model="beta", bdraw="exact (Cholesky + SVD-floor rule)")


if __name__ == "__main__":
    main()
