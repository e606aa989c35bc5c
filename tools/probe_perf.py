"""Quick GPU timing probe: sweeps/s of the sweep kernel at several chain counts (and
waves per chain)."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from gibbs_student_t_amd import data  # noqa: E402
from gibbs_student_t_amd.model import PTA  # noqa: E402
from gibbs_student_t_amd.native import NativeSampler  # noqa: E402


def main():
    psr = data.j1713()
    pta = PTA(psr)
    cfg = dict(model="mixture", vary_df=True, theta_prior="beta")
    # arguments: C or C:waves (waves per chain: 1, 2; default auto)
    for arg in (sys.argv[1:] or ["256", "1024", "2048"]):
        C, _, w = arg.partition(":")
        C = int(C)
        ns = NativeSampler(pta, cfg, 0)
        ns.set_waves(int(w) if w else "auto")
        ns.alloc(C)
        rng = np.random.default_rng(0)
        x0 = np.stack([[rng.uniform(1, 7), rng.uniform(-18, -12), rng.uniform(-10, -5)]
                       for _ in range(C)])
        ns.set_state(x=x0, z=np.ones((C, ns.n)), alpha=np.ones((C, ns.n)),
                     theta=np.full(C, 0.01), nu=np.full(C, 4.0))
        ns.sweep(20, seed=1)
        ns.synchronize()
        S = 100
        rec = ns.alloc_records(S)
        t0 = time.perf_counter()
        ns.sweep(S, records=rec, seed=1, sweep0=20)
        ns.synchronize()
        dt = time.perf_counter() - t0
        kms = ns.last_kernel_ms()
        st = ns.get_state()
        print(f"C={C} waves={w or 'auto'} sweeps={S} wall={dt*1e3:.1f} ms kernel={kms:.1f} ms  "
              f"-> {C*S/dt:.3e} chain-sweeps/s, {dt/S*1e6:.1f} us/sweep; "
              f"status!=0: {(st['status']!=0).sum()}", flush=True)
        ns.close()


if __name__ == "__main__":
    main()
