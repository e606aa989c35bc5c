"""The notebook's own run at its own size, on the large path (missing 1).

gibbs_likelihood.ipynb runs J1643-1224 (12,863 TOAs, ipynb:60-61,711) under one efac, equad
and ECORR (no_selection), 20 red-noise components and the timing model (cell 2), model
'vvh17' (cell 4), at 18.9 sweeps/s on one CPU chain.  The data are not in the
reference, so this builds a synthetic pulsar of that shape with the simulate_data recipe
(data.multiband: 130 J1713+0747 epochs x 99 sub-band TOAs = 12,870 TOAs, one ECORR epoch per
observation) and times chain-sweeps on the large path, with the structured ECORR Gram
(lg_gram_ec, the default) and with the dense one (GST_DEBUG_LARGE_GRAM).

    python tools/j1643_rate.py [chains] [sweeps]
    python tools/j1643_rate.py --cpu [seconds]   # the reference algorithm on one CPU core

(--cpu: oracle/gibbs_oracle.py, the line-cited restatement of gibbs.py that reproduces its
chains bit for bit, with numpy's legacy RNG calls -- as the test-infrastructure CPU baseline.)
"""
import json
import sys

import numpy as np

sys.path.insert(0, ".")
from gibbs_student_t_amd import data  # noqa: E402
from gibbs_student_t_amd.model import PTA  # noqa: E402
from gibbs_student_t_amd.native import NativeSampler  # noqa: E402
from gibbs_student_t_amd.run_sims import MODELS  # noqa: E402


def j1643_like():
    psr = data.multiband(nepochs=130, nsub=99, seed=1643, components=20)
    return PTA(psr, components=20, efac=(0.2, 10.0), log10_equad=(-10.0, -5.0),
               log10_A=(-18.0, -12.0), gamma=(0.0, 7.0), log10_ecorr=(-8.0, -5.0),
               ecorr_dt=30.0)


def rate(pta, C, S, **debug):
    ns = NativeSampler(pta, MODELS["vvh17"], 0, path="large")
    ns.set_debug(**debug)
    ns.alloc(C)
    rng = np.random.default_rng(3)
    lo = np.array([p.pmin for p in pta.params])
    hi = np.array([p.pmax for p in pta.params])
    ns.set_state(x=rng.uniform(lo, hi, size=(C, len(lo))), z=np.ones((C, ns.n)),
                 alpha=np.full((C, ns.n), 1e10), theta=np.full(C, 0.05), nu=np.full(C, 4.0))
    ns.sweep(3, seed=1)
    ns.set_timing(True)
    ns.sweep(S, seed=1, sweep0=3)
    ns.synchronize()
    kt = ns.kernel_times()
    ms = sum(v[0] for v in kt.values())
    st = ns.get_state()["status"]
    ns.close()
    return {"chains": C, "sweeps": S, "chain_sweeps_per_s": C * S / (ms * 1e-3),
            "ms_per_sweep": ms / S, "stages_ms_per_sweep": {k: v[0] / S for k, v in kt.items()},
            "status_clean": bool(np.all((st & 0xef) == 0))}


def cpu_rate(seconds):
    import os
    import time
    import warnings
    os.environ.setdefault("OPENBLAS_NUM_THREADS", "1")
    from oracle.gibbs_oracle import LegacyNumpyVariates, Oracle, OutlierModel, initial_state
    warnings.simplefilter("ignore")
    pta = j1643_like()
    orc = Oracle(pta, OutlierModel(**MODELS["vvh17"]))
    st = initial_state(pta, orc.cfg)
    np.random.seed(5)
    x = np.array(pta.sample_params(), dtype=np.float64)
    src = LegacyNumpyVariates()
    x = orc.sweep(st, x, src)    # (first sweep: caches and page-in)
    t0, k = time.perf_counter(), 0
    while time.perf_counter() - t0 < seconds:
        x = orc.sweep(st, x, src)
        k += 1
    dt = time.perf_counter() - t0
    return {"dataset": "j1643-like", "cpu": "oracle (reference algorithm), 1 core",
            "sweeps": k, "seconds": dt, "sweeps_per_s": k / dt}


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--cpu":
        print(json.dumps(cpu_rate(float(sys.argv[2]) if len(sys.argv) > 2 else 20.0)))
        return
    C = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    S = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    pta = j1643_like()
    shape = {"n": pta.n, "m": pta.m, "n_ecorr": int(len(pta.ecorr_backend)),
             "params": [p.name for p in pta.params]}
    print(json.dumps({"dataset": "j1643-like", **shape}), flush=True)
    for label, dbg in (("structured ECORR Gram", {}), ("dense Gram", {"large_gram": True})):
        r = rate(pta, C, S, **dbg)
        print(json.dumps({"gram": label, **r}), flush=True)


if __name__ == "__main__":
    main()
