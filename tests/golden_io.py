"""Load the golden fixtures (tests/golden/*.npz, made by tools/gen_golden.py)."""
from __future__ import annotations

import ast
import glob
import os

import numpy as np

from gibbs_student_t_amd.model import PTA

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

CHAIN_KEYS = ("chain", "bchain", "zchain", "poutchain", "thetachain", "alphachain", "dfchain")


def fixture_names():
    return sorted(os.path.basename(p)[4:-4] for p in glob.glob(os.path.join(GOLDEN, "ref_*.npz")))


def load_dataset(efac=False, dataset="j1713"):
    fn = "j1713_dataset_efac.npz" if efac else f"{dataset}_dataset.npz"
    d = np.load(os.path.join(GOLDEN, fn), allow_pickle=False)
    return PTA.from_arrays("J1713+0747", d["residuals"], d["toaerrs"], d["T"], d["Ffreqs"],
                           int(d["components"]), float(d["tm_weight"]),
                           efac=(0.2, 10.0) if efac else 1.0)


def load_ref(name):
    d = dict(np.load(os.path.join(GOLDEN, f"ref_{name}.npz"), allow_pickle=False))
    d["kw"] = ast.literal_eval(str(d.pop("model_kw")))
    d["tape"] = {k[5:]: v for k, v in d.items() if k.startswith("tape_")}
    ds = name.split("_")[0] if name.split("_")[0] in ("sim", "twob", "simclean", "scaled") else "j1713"
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
