"""KS p-values of 1024 GPU chains against the reference's posterior draws
(tests/golden/posterior_ref_<dataset>_beta.npz), per path variant, for the record:

    python tools/ks_diag_gen.py <dataset> [persistent,persistent_mfma,large,large_generic]
"""
import os, sys
import numpy as np, scipy.stats
sys.path.insert(0, "."); sys.path.insert(0, "tests")
from golden_io import GOLDEN, load_dataset
from gibbs_student_t_amd.native import NativeSampler
from gibbs_student_t_amd.run_sims import MODELS
ds = sys.argv[1]
ref = np.load(os.path.join(GOLDEN, f"posterior_ref_{ds}_beta.npz"), allow_pickle=False)
burn, thin = int(ref["burn"]), 2 * int(ref["thin"])
rx, rth, rnu = ref["x"][:, ::2], ref["theta"][:, ::2], ref["nu"][:, ::2]
pta = load_dataset(dataset=ds)
# variants: argv[2], comma-separated (default: both paths and the MFMA-Gram persistent build;
# "large_generic": the large path with GST_DEBUG_LARGE_HYPER, e.g. mb's lg_hyper<0>)
for variant in (sys.argv[2].split(",") if len(sys.argv) > 2 else ("persistent", "persistent_mfma", "large")):
    path = "large" if variant.startswith("large") else "persistent"
    C, S = 1024, burn + 60 * thin
    ns = NativeSampler(pta, MODELS["beta"], 0, path=path)
    if variant == "persistent_mfma":
        ns.set_debug(mfma_gram=True)
    if variant == "large_generic":
        ns.set_debug(large_hyper=True)
    ns.alloc(C)
    lo = np.array([p.pmin for p in pta.params]); hi = np.array([p.pmax for p in pta.params])
    ns.set_state(x=np.random.default_rng(6).uniform(lo, hi, size=(C, len(lo))), z=np.ones((C, pta.n)),
                 alpha=np.ones((C, pta.n)), theta=np.full(C, 0.01), nu=np.full(C, 4.0))
    ns.sweep(burn, seed=78)
    rec = ns.alloc_records(S - burn, keys=("x", "theta", "nu"))
    ns.sweep(S - burn, records=rec, seed=78, sweep0=burn)
    got = {k: v.cpu().numpy()[:, ::thin] for k, v in rec.items()}
    ns.close()
    names = [str(s) for s in ref["names"]]
    out = []
    for j, nm in enumerate(names):
        out.append((nm[-12:], scipy.stats.ks_2samp(got["x"][..., j].ravel(), rx[..., j].ravel()).pvalue))
    out.append(("theta", scipy.stats.ks_2samp(got["theta"].ravel(), rth.ravel()).pvalue))
    out.append(("nu", scipy.stats.ks_2samp(got["nu"].ravel(), rnu.ravel()).pvalue))
    print(ds, variant, "theta mean %.5f (ref %.5f) nu mean %.3f (ref %.3f)" % (got["theta"].mean(), rth.mean(), got["nu"].mean(), rnu.mean()),
          " ".join("%s:%.1e" % (a, b) for a, b in out), flush=True)
