"""Per-dataset convergence of BASELINE config 4.

    python tools/config4_rhat.py [out.json] [worst.npz] [--save D1,D2,...] [--exact]
        [--chains PER_DATASET] [--seed S]

Runs bench.py's config-4 workload (256 run_sims datasets x 64 chains on one GPU) with the
bench's own schedule (300 warmup sweeps, 1000 timed, 3000 burn-in, then a 5000-sweep window
recorded every 5th sweep), computes rank-normalised split-R-hat and bulk-ESS PER DATASET
for every sampled parameter and theta, and writes every dataset's row (model, kind,
theta_sim, dof, n, R-hats) sorted by the worst R-hat.  The window draws of the worst
mixture-model ('beta' / 'uniform') dataset are saved so that tools/config4_oracle.py can
compare them with the reference algorithm (the oracle) run on the same dataset; ``--save``
also saves the listed datasets' window draws (<worst stem>_d<D>.npz) for
tools/config4_same_start.py.  The chains start as bench.workload starts them (prior draws,
gibbs.py:29-51 latents, vvh17 at the reference's z = 1).  ``--exact``: no SVD noise floor
in the b draw (GST_DEBUG_EXACT_BDRAW).
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from gibbs_student_t_amd import diag, run_sims  # noqa: E402
from gibbs_student_t_amd.native import NativeSampler  # noqa: E402

W, K, BURN, WIN, THIN, SEED = 300, 1000, 3000, 5000, 5, 20171713


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    save, chains, seed = [], None, SEED
    for i, a in enumerate(sys.argv):
        if a == "--save":
            save = [int(v) for v in sys.argv[i + 1].split(",")]
            args.remove(sys.argv[i + 1])
        if a == "--chains":        # chains per dataset (default 64, the bench's)
            chains = int(sys.argv[i + 1])
            args.remove(sys.argv[i + 1])
        if a == "--seed":
            seed = int(sys.argv[i + 1])
            args.remove(sys.argv[i + 1])
    dst = args[0] if len(args) > 0 else "config4_rhat.json"
    worst_npz = args[1] if len(args) > 1 else None
    wl = bench.workload(4, 0, 1, chains)
    grid = run_sims.build_grid(thetas=(0.05, 0.1, 0.15), realisations=5,
                               dofs=(None, 4.0))[:bench.CONFIG4_DATASETS]
    ns = NativeSampler(wl["ptas"], wl["cfgs"], 0)
    ns.alloc(wl["C"], dataset=wl["ds"])
    ns.set_debug(exact_bdraw="--exact" in sys.argv)
    ns.set_state(**wl["init"])
    ns.sweep(W + K + BURN, seed=seed, sweep0=0, chain0=0)
    rec = ns.alloc_records(WIN // THIN, keys=("x", "theta"))
    ns.sweep(WIN, records=rec, record_every=THIN, seed=seed, sweep0=W + K + BURN, chain0=0)
    x = rec["x"].cpu().numpy()
    th = rec["theta"].cpu().numpy()
    z = ns.get_state()["z"]
    ns.close()
    names = [p.name.split("_", 1)[1] for p in wl["ptas"][0].params]
    rows = []
    for d, e in enumerate(grid):
        sel = wl["ds"] == d
        row = {"dataset": d, "model": e.model, "kind": e.kind, "theta_sim": e.theta,
               "dof": e.dof, "n": e.pta.n, "n_outliers_true": int(e.meta["z_true"].sum()),
               "mean_sum_z_end": float(z[sel][:, :e.pta.n].sum(1).mean())}
        series = {nm: x[sel, :, j] for j, nm in enumerate(names)}
        if e.cfg["model"] in ("mixture", "vvh17"):
            series["theta"] = th[sel]
        rh = {}
        for nm, v in series.items():
            ess, r = diag.ess_rhat(v)
            rh[nm] = float(r)
            row[f"ess_{nm}"] = float(ess)
        row["rhat"] = rh
        row["rhat_max"] = max(rh.values())
        # per-chain means of the worst parameter: a multimodal posterior shows as clusters
        worst = max(rh, key=rh.get)
        row["worst_param"] = worst
        row["chain_means_worst"] = np.sort(series[worst].mean(axis=1)).round(5).tolist()
        rows.append(row)
    rows.sort(key=lambda r: -r["rhat_max"])
    by_model = {}
    for r in rows:
        b = by_model.setdefault(r["model"], {"datasets": 0, "rhat_gt_1.01": 0, "worst": 0.0})
        b["datasets"] += 1
        b["rhat_gt_1.01"] += int(r["rhat_max"] > 1.01)
        b["worst"] = max(b["worst"], r["rhat_max"])
    out = {"schedule": {"warmup": W, "timed": K, "burn": BURN, "window": WIN, "thin": THIN,
                        "seed": seed, "chains_per_dataset": wl["per"]},
           "start": "bench.workload(4): prior draws, gibbs.py:29-51 latents (vvh17 z = 1)",
           "b_draw": "exact" if "--exact" in sys.argv else "SVD noise floor (include/gst.h)",
           "by_model": by_model, "datasets": rows}
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    for r in rows[:25]:
        print(json.dumps({k: r[k] for k in ("dataset", "model", "kind", "theta_sim", "dof", "n",
                                            "n_outliers_true", "rhat_max", "worst_param",
                                            "mean_sum_z_end")}))
    print(json.dumps(by_model))
    if worst_npz:
        # the worst 'beta' and the worst 'uniform' dataset, and every --save dataset:
        # <stem>_d<dataset>.npz each
        stem = worst_npz[:-4] if worst_npz.endswith(".npz") else worst_npz
        picks = list(save)
        for mdl in ("beta", "uniform"):
            mix = [r for r in rows if r["model"] == mdl]
            if mix:
                picks.append(mix[0]["dataset"])
        for d in dict.fromkeys(picks):
            sel = wl["ds"] == d
            np.savez(f"{stem}_d{d}.npz", dataset=d, x=x[sel], theta=th[sel],
                     names=np.array(names), thin=THIN, first_sweep=W + K + BURN)
            print("dataset", d, "saved to", f"{stem}_d{d}.npz")


if __name__ == "__main__":
    main()
