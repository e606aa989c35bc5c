"""ecq (GEN model, small nu) theta / nu window means against burn-in length: does the GPU's
posterior drift with the window (slow mixing) or stay put?  python tools/ks_burnin_gen.py"""
import os
import sys

import numpy as np

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from golden_io import GOLDEN, load_dataset  # noqa: E402
from gibbs_student_t_amd.native import NativeSampler  # noqa: E402
from gibbs_student_t_amd.run_sims import MODELS  # noqa: E402

ds = sys.argv[1] if len(sys.argv) > 1 else "ecq"
pta = load_dataset(dataset=ds)
ref = np.load(os.path.join(GOLDEN, f"posterior_ref_{ds}_beta.npz"), allow_pickle=False)
print("reference theta mean %.5f (8 chains: %s)" % (ref["theta"].mean(),
      np.round(ref["theta"].mean(1), 4)))
C = 1024
ns = NativeSampler(pta, MODELS["beta"], 0)
ns.alloc(C)
lo = np.array([p.pmin for p in pta.params])
hi = np.array([p.pmax for p in pta.params])
ns.set_state(x=np.random.default_rng(6).uniform(lo, hi, size=(C, len(lo))), z=np.ones((C, pta.n)),
             alpha=np.ones((C, pta.n)), theta=np.full(C, 0.01), nu=np.full(C, 4.0))
done = 0
for w in range(8):
    S = 3000
    rec = ns.alloc_records(S, keys=("theta", "nu"))
    ns.sweep(S, records=rec, seed=78, sweep0=done)
    done += S
    th = rec["theta"].cpu().numpy()
    nu = rec["nu"].cpu().numpy()
    print("sweeps %6d-%6d theta mean %.5f nu mean %.3f  chain-mean sd %.5f" %
          (done - S, done, th.mean(), nu.mean(), th.mean(axis=1).std()), flush=True)
