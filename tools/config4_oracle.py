"""Is config 4's slow convergence the posterior or the kernel?  

    OPENBLAS_NUM_THREADS=1 python tools/config4_oracle.py DATASET [gpu_window.npz] [out.json]

Runs the oracle (oracle/gibbs_oracle.py: the reference algorithm, bit-exact to gibbs.py
with numpy's legacy RNG) on one dataset of bench.py's config-4 grid (run_sims.build_grid,
host generator, the same seeded datasets the GPU samples) with 8 chains from prior draws,
one process each, on the bench's schedule: 4300 discarded sweeps (bench warmup + timed +
ESS burn-in), then a 5000-sweep window recorded every 5th sweep.  Prints the oracle's
split-R-hat / bulk-ESS and per-chain means next to the GPU window's (from
tools/config4_rhat.py's npz when given), and two-sample KS p-values between the pooled
oracle and GPU draws.  If the reference algorithm's chains show the same between-chain
spread, the R-hat is the posterior's (multimodality / slow mixing), not the kernel's.
"""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

BURN, WIN, THIN, CHAINS = 4300, 5000, 5, 8


def grid_entry(d):
    import bench
    from gibbs_student_t_amd import run_sims
    grid = run_sims.build_grid(thetas=(0.05, 0.1, 0.15), realisations=5,
                               dofs=(None, 4.0))[:bench.CONFIG4_DATASETS]
    return grid[d]


def worker(d, seed, out):
    import warnings
    from oracle.gibbs_oracle import (LegacyNumpyVariates, Oracle, OutlierModel,
                                     initial_state)
    warnings.simplefilter("ignore")
    e = grid_entry(d)
    orc = Oracle(e.pta, OutlierModel(**e.cfg))
    np.random.seed(seed)
    x = e.pta.sample_params()
    st = initial_state(e.pta, orc.cfg)
    src = LegacyNumpyVariates()
    rec = []
    for i in range(BURN + WIN):
        if i >= BURN and (i - BURN) % THIN == 0:
            rec.append(list(x) + [float(st.theta)])   # state at the start of the sweep
        x = orc.sweep(st, x, src)
    np.save(out, np.asarray(rec))


def main():
    if sys.argv[1] == "--worker":
        worker(int(sys.argv[2]), int(sys.argv[3]), sys.argv[4])
        return
    import scipy.stats
    from gibbs_student_t_amd import diag
    d = int(sys.argv[1])
    gpu = np.load(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[2] != "-" else None
    dst = sys.argv[3] if len(sys.argv) > 3 else None
    e = grid_entry(d)
    names = [p.name.split("_", 1)[1] for p in e.pta.params] + ["theta"]
    env = dict(os.environ, OPENBLAS_NUM_THREADS="1", OMP_NUM_THREADS="1")
    with tempfile.TemporaryDirectory() as td:
        outs = [os.path.join(td, f"c{i}.npy") for i in range(CHAINS)]
        procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__), "--worker",
                                   str(d), str(4000 + i), outs[i]], env=env)
                 for i in range(CHAINS)]
        for p in procs:
            p.wait()
        orc = np.stack([np.load(o) for o in outs])          # [chains, draws, P + 1]
    res = {"dataset": d, "model": e.model, "kind": e.kind, "theta_sim": e.theta, "dof": e.dof,
           "n": e.pta.n, "schedule": {"burn": BURN, "window": WIN, "thin": THIN},
           "oracle_chains": CHAINS, "params": {}}
    for j, nm in enumerate(names):
        o = orc[:, :, j]
        ess, rh = diag.ess_rhat(o)
        row = {"oracle_rhat": float(rh), "oracle_ess": float(ess),
               "oracle_chain_means": np.sort(o.mean(1)).round(5).tolist()}
        if gpu is not None:
            g = gpu["x"][:, :, j] if j < len(names) - 1 else gpu["theta"]
            gess, grh = diag.ess_rhat(g)
            row.update({"gpu_rhat": float(grh), "gpu_ess": float(gess),
                        "gpu_chain_mean_quantiles": np.quantile(g.mean(1), [0, .1, .5, .9, 1])
                        .round(5).tolist(),
                        "ks_p_oracle_vs_gpu": float(scipy.stats.ks_2samp(
                            o[:, ::2].ravel(), g[:, ::2].ravel()).pvalue)})
        res["params"][nm] = row
        print(nm, json.dumps(row), flush=True)
    if dst:
        with open(dst, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
