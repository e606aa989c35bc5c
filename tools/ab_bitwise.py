"""Are two libgst builds' chains bitwise identical?  (A kernel change that claims to be
semantics-neutral, e.g. the paired elimination tail, must leave every draw unchanged.)

    python tools/ab_bitwise.py LIB_A LIB_B [chains] [sweeps]

Each library runs in its own process (GST_LIB) from the same prior-draw start, on the
J1713+0747 headline workload and on the config-3 / 20-component / 22-TM-column fixtures'
datasets, recording every sweep; the records and final states are compared bitwise.
AB_CASES picks the cases (also syn<N>k: a scaled synthetic pulsar of N thousand TOAs), AB_PATH
the sampler path (auto / persistent / large).
"""
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = ("x", "b", "z", "alpha", "pout", "theta", "nu")
CASES = tuple(os.environ.get("AB_CASES", "j1713,c3,c20,tm22").split(","))


def worker(case, C, S, out):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from golden_io import load_dataset
    from gibbs_student_t_amd.native import NativeSampler
    cfg = dict(model="mixture", vary_df=True, theta_prior="beta")
    if case.startswith("syn"):        # scaled synthetic pulsar, n = syn<N>k TOAs (large path)
        from gibbs_student_t_amd import data
        from gibbs_student_t_amd.model import PTA
        n = int(case[3:].rstrip("k")) * 1000
        pta = PTA(data.scaled_synthetic(n=n, components=30, ntm=50, seed=5), components=30)
    else:
        pta = load_dataset(dataset=case) if case != "j1713" else load_dataset()
    ns = NativeSampler(pta, cfg, 0, path=os.environ.get("AB_PATH", "auto"))
    ns.alloc(C)
    lo = np.array([p.pmin for p in pta.params])
    hi = np.array([p.pmax for p in pta.params])
    ns.set_state(x=np.random.default_rng(3).uniform(lo, hi, size=(C, len(lo))),
                 z=np.ones((C, ns.n)), alpha=np.ones((C, ns.n)), theta=np.full(C, 0.01),
                 nu=np.full(C, 4.0))
    # per-TOA records only for small pulsars (C x S x n doubles each)
    rec = ns.alloc_records(S, keys=("x", "b", "theta", "nu")) if ns.n > 4096 else \
        ns.alloc_records(S)
    ns.sweep(S, records=rec, seed=99)
    fin = ns.get_state()
    np.savez(out, **{f"rec_{k}": v.cpu().numpy() for k, v in rec.items()},
             **{f"fin_{k}": v for k, v in fin.items()})
    ns.close()


def main():
    if sys.argv[1] == "--worker":
        worker(sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), sys.argv[5])
        return 0
    a, b = sys.argv[1], sys.argv[2]
    C = int(sys.argv[3]) if len(sys.argv) > 3 else 2048
    S = int(sys.argv[4]) if len(sys.argv) > 4 else 60
    ok = True
    with tempfile.TemporaryDirectory() as td:
        for case in CASES:
            outs = []
            for lib in (a, b):
                out = os.path.join(td, f"{case}_{os.path.basename(lib)}.npz")
                env = dict(os.environ, GST_LIB=os.path.abspath(lib))
                subprocess.run([sys.executable, os.path.abspath(__file__), "--worker", case,
                                str(C), str(S), out], env=env, check=True)
                outs.append(np.load(out))
            bad = [k for k in outs[0].files if not np.array_equal(outs[0][k], outs[1][k])]
            print(f"{case}: {'bitwise identical' if not bad else 'DIFFER in ' + ', '.join(bad)}",
                  flush=True)
            ok = ok and not bad
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
