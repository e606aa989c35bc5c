"""Load the golden fixtures (tests/golden/*.npz, made by tools/gen_golden.py)."""
from __future__ import annotations

import ast
import glob
import os

import numpy as np

from gibbs_student_t_amd.model import PTA

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

# fixture-name prefix -> tests/golden/{prefix}_dataset.npz (tools/gen_golden.py)
DATASETS = ("sim", "twob", "simclean", "scaled", "c3", "c4t", "c20", "tm22", "mb", "mbn",
            "mid", "wide", "ecb", "ecn", "ecq", "ebig", "jb")

CHAIN_KEYS = ("chain", "bchain", "zchain", "poutchain", "thetachain", "alphachain", "dfchain")


def fixture_names():
    return sorted(os.path.basename(p)[4:-4] for p in glob.glob(os.path.join(GOLDEN, "ref_*.npz")))


def load_dataset(efac=False, dataset="j1713"):
    fn = "j1713_dataset_efac.npz" if efac else f"{dataset}_dataset.npz"
    d = np.load(os.path.join(GOLDEN, fn), allow_pickle=False)
    if "backends" in d.files:     # general white-noise model (tools/gen_golden.py general)
        name = str(d["names"][0]).split("_")[0]
        return PTA.from_arrays(name, d["residuals"], d["toaerrs"], d["T"], d["Ffreqs"],
                               int(d["components"]), float(d["tm_weight"]),
                               efac=(0.2, 10.0) if int(d["efac_varied"]) else 1.0,
                               backends=d["backends"], selection=str(d["selection"]),
                               n_ecorr=int(d["n_ecorr"]), ecorr_backend=d["ecorr_backend"],
                               log10_ecorr=tuple(d["log10_ecorr"]) or None)
    return PTA.from_arrays("J1713+0747", d["residuals"], d["toaerrs"], d["T"], d["Ffreqs"],
                           int(d["components"]), float(d["tm_weight"]),
                           efac=(0.2, 10.0) if efac else 1.0)


def load_ref(name):
    d = dict(np.load(os.path.join(GOLDEN, f"ref_{name}.npz"), allow_pickle=False))
    d["kw"] = ast.literal_eval(str(d.pop("model_kw")))
    d["tape"] = {k[5:]: v for k, v in d.items() if k.startswith("tape_")}
    ds = name.split("_")[0] if name.split("_")[0] in DATASETS else "j1713"
    d["pta"] = load_dataset(efac="efac" in name, dataset=ds)
    return d


def sweep_state(ref, i):
    """State at the START of sweep i (i == niter -> the final state)."""
    niter = int(ref["niter"])
    if i < niter:
        return dict(x=ref["chain"][i], b=ref["bchain"][i], z=ref["zchain"][i],
                    alpha=ref["alphachain"][i], pout=ref["poutchain"][i],
                    theta=float(ref["thetachain"][i]), nu=float(ref["dfchain"][i]))
    return dict(x=None, b=ref["final_b"], z=ref["final_z"], alpha=ref["final_alpha"],
                pout=ref["final_pout"], theta=float(ref["final_theta"]),
                nu=float(ref["final_df"]))


def sweep_tape(ref, i):
    return {k: v[i] for k, v in ref["tape"].items()}


def oracle_replay(ref, S=None):
    """The oracle replaying the reference's tape for S sweeps from the recorded start with
    the Cholesky mean and the recorded draw term (b = cho_solve(Sigma, d) + b_delta,
    gibbs.py:321-322 + 169-180; at the SVD noise floor, Sigma beyond fp64 resolution, the
    mean of Sigma + f I: Oracle.floor_shift).  That is the expression the HIP path evaluates
    in tape mode, so the two chains agree to fp64 rounding, not to the SVD-vs-Cholesky mean
    gap that separates both from the reference's own chain.  Returns records {key: [S, ...]}
    of the state at the start of each sweep (gibbs.py:355-361)."""
    import warnings

    from oracle.gibbs_oracle import ChainState, Oracle, OutlierModel, TapeVariates
    S = int(ref["niter"]) if S is None else int(S)
    orc = Oracle(ref["pta"], OutlierModel(**ref["kw"]))
    s0 = sweep_state(ref, 0)
    st = ChainState(b=s0["b"].copy(), z=s0["z"].copy(), alpha=s0["alpha"].copy(),
                    pout=s0["pout"].copy(), theta=s0["theta"], nu=s0["nu"])
    x = np.array(ref["xs"], dtype=np.float64)
    rec = {k: [] for k in ("x", "b", "z", "alpha", "pout", "theta", "nu")}
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        for i in range(S):
            for k, v in (("x", x), ("b", st.b), ("z", np.asarray(st.z, float)),
                         ("alpha", st.alpha), ("pout", st.pout), ("theta", st.theta),
                         ("nu", float(st.nu))):
                rec[k].append(np.array(v, dtype=np.float64, copy=True))
            x = orc.sweep(st, x, TapeVariates(sweep_tape(ref, i)), b_mean="floor_delta")
    return {k: np.stack(v) for k, v in rec.items()}
