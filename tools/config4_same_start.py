"""Config-4 distributional parity from the same start.

    OPENBLAS_NUM_THREADS=1 python tools/config4_same_start.py oracle D VARIANT OUT.npz [NCHAINS]
    python tools/config4_same_start.py compare D GPU.npz ORACLE_SVD.npz [ORACLE_FLOOR.npz] OUT.json

``oracle``: the reference algorithm (oracle/gibbs_oracle.py with gibbs.py's legacy RNG calls)
on dataset D of bench.py's config-4 grid, NCHAINS (64) chains from EXACTLY the initial states
of the GPU chains of ``config4_rhat.py --chains NCHAINS`` (run_sims.initial_state(entry,
NCHAINS, NCHAINS D, 7, ...): the prior draws and gibbs.py:29-51
latents bench.workload gives them, vvh17 at the reference's z = 1), on the bench schedule
(4300 sweeps, then a 5000-sweep window recorded every 5th sweep).  VARIANT ``svd`` is the
reference's own b draw (gibbs.py:169-180); ``floor`` the HIP path's rule (exact draw, at the
SVD noise floor from Sigma + f I; Oracle.floor_shift).  One process per chain slot (8).

``compare``: per-chain modes (the two clusters of the window-mean log10_equad split at the
largest gap; vvh17's all-outlier state counted too), a Fisher exact test of the mode counts
GPU vs oracle, KS and Welch t tests of the per-chain window means within each mode (the
chains are the independent samples), and split-R-hat of each sample.  The GPU draws come
from tools/config4_rhat.py (``--save D1,D2,...``).
"""
import json
import os
import sys
import warnings
from multiprocessing import Pool

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

BURN, WIN, THIN, CHAINS, SEED0 = 4300, 5000, 5, 64, 7


def _entry(d):
    import bench
    from gibbs_student_t_amd import run_sims
    grid = run_sims.build_grid(thetas=(0.05, 0.1, 0.15), realisations=5,
                               dofs=(None, 4.0))[:bench.CONFIG4_DATASETS]
    return grid[d]


def _chain(args):
    d, variant, c, nch = args
    warnings.simplefilter("ignore")
    from gibbs_student_t_amd import run_sims
    from oracle.gibbs_oracle import ChainState, LegacyNumpyVariates, Oracle, OutlierModel
    e = _entry(d)
    n = e.pta.n
    # bench.workload(4, chains=nch) gives dataset d the chain ids d*nch .. d*nch + nch - 1
    init = run_sims.initial_state(e, nch, d * nch, SEED0, n, "reference")
    orc = Oracle(e.pta, OutlierModel(**e.cfg))
    st = ChainState(b=init["b"][c].copy(), z=init["z"][c, :n].copy(),
                    alpha=init["alpha"][c, :n].copy(), pout=init["pout"][c, :n].copy(),
                    theta=float(init["theta"][c]), nu=float(init["nu"][c]))
    x = init["x"][c].copy()
    np.random.seed(90000 + 1000 * d + c)
    src = LegacyNumpyVariates()
    mean = "svd" if variant == "svd" else "floor"
    rec = []
    for i in range(BURN + WIN):
        if i >= BURN and (i - BURN) % THIN == 0:
            rec.append(list(x) + [float(st.theta)])   # state at the start of the sweep
        x = orc.sweep(st, x, src, b_mean=mean)
    return np.asarray(rec), float(np.sum(st.z))


def run_oracle(d, variant, out, nch=CHAINS):
    """NCHAINS chains starting exactly as the GPU's config4_rhat.py --chains NCHAINS."""
    with Pool(8) as pool:
        res = pool.map(_chain, [(d, variant, c, nch) for c in range(nch)], chunksize=1)
    e = _entry(d)
    names = [p.name.split("_", 1)[1] for p in e.pta.params]
    np.savez(out, dataset=d, variant=variant, x=np.stack([r[0][:, :-1] for r in res]),
             theta=np.stack([r[0][:, -1] for r in res]),
             sum_z_end=np.array([r[1] for r in res]), names=np.array(names), thin=THIN,
             first_sweep=BURN)


def compare(d, gpu_f, svd_f, floor_f, out):
    import scipy.stats
    from gibbs_student_t_amd import diag
    e = _entry(d)
    samples = {"gpu": np.load(gpu_f), "oracle_svd": np.load(svd_f)}
    if floor_f:
        samples["oracle_floor"] = np.load(floor_f)
    names = [str(s) for s in samples["oracle_svd"]["names"]]
    res = {"dataset": d, "model": e.model, "kind": e.kind, "theta_sim": e.theta, "dof": e.dof,
           "n": e.pta.n, "schedule": {"burn": BURN, "window": WIN, "thin": THIN},
           "start": "run_sims.initial_state(..., 'reference'): the GPU chains' own states",
           "samples": {}}
    # modes: the pooled chain means of log10_equad split at their largest gap (the bimodal
    # posteriors of config 4: outliers flagged vs absorbed into a large EQUAD); vvh17's
    # all-outlier state (window-mean theta >= 1/2) is counted separately
    j = [i for i, nm in enumerate(names) if "equad" in nm][0]
    cm = np.sort(np.concatenate([s["x"][:, :, j].mean(1) for s in samples.values()]))
    gaps = np.diff(cm)
    g = int(np.argmax(gaps))
    cut = 0.5 * (cm[g] + cm[g + 1])
    res["mode_rule"] = f"window-mean {names[j]} > {cut:.4f} (largest gap {gaps[g]:.3f})"
    lab = {k: (s["x"][:, :, j].mean(1) > cut).astype(int) for k, s in samples.items()}
    series = lambda s: [(nm, s["x"][:, :, i]) for i, nm in enumerate(names)] + \
        [("theta", s["theta"])]
    for k, s in samples.items():
        row = {"mode1_chains": int(lab[k].sum()), "chains": int(len(lab[k])),
               "all_outlier_chains": int(np.sum(s["theta"].mean(1) >= 0.5)), "rhat": {}}
        for nm, v in series(s):
            row["rhat"][nm] = float(diag.ess_rhat(v)[1])
        res["samples"][k] = row
    # Within a mode the draws of a chain are autocorrelated (a pooled KS of 64 x 1000 draws
    # rejects even between two runs of the reference algorithm), so the chains are the
    # independent samples: KS and Welch t on the per-chain window means, per mode.
    for k in samples:
        if k == "oracle_svd":
            continue
        a, b = lab[k], lab["oracle_svd"]
        table = [[int(a.sum()), int(len(a) - a.sum())], [int(b.sum()), int(len(b) - b.sum())]]
        cmp = {"mode_table": table, "fisher_p": float(scipy.stats.fisher_exact(table)[1]),
               "chain_means_in_mode": {}}
        for (nm, gx), (_, rx) in zip(series(samples[k]), series(samples["oracle_svd"])):
            for m in (0, 1):
                gm, rm = gx[a == m].mean(1), rx[b == m].mean(1)
                if len(gm) >= 3 and len(rm) >= 3:
                    cmp["chain_means_in_mode"].setdefault(f"mode{m}", {})[nm] = {
                        "ks_p": float(scipy.stats.ks_2samp(gm, rm).pvalue),
                        "welch_p": float(scipy.stats.ttest_ind(gm, rm, equal_var=False).pvalue)}
        res[f"{k}_vs_oracle_svd"] = cmp
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


def main():
    if sys.argv[1] == "oracle":
        run_oracle(int(sys.argv[2]), sys.argv[3], sys.argv[4],
                   int(sys.argv[5]) if len(sys.argv) > 5 else CHAINS)
    elif sys.argv[1] == "compare":
        rest = sys.argv[3:]
        floor_f = rest[2] if len(rest) == 4 else None
        compare(int(sys.argv[2]), rest[0], rest[1], floor_f, rest[-1])
    else:
        raise SystemExit(__doc__)


if __name__ == "__main__":
    main()
