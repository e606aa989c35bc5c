"""Stage costs of the persistent kernel from stage-masked launches (no stamp overhead).

    python tools/stage_mask_timing.py [C] [S] [j1713|c3]

Times S sweeps of C chains (J1713+0747, or bench config 3's simulated pulsar) for several
stage masks (gst_sweep stage_mask) and prints the per-sweep kernel time of each and the
differences (a stage's marginal cost).
"""
import sys

import numpy as np

sys.path.insert(0, ".")
from gibbs_student_t_amd import _abi, data  # noqa: E402
from gibbs_student_t_amd.model import PTA  # noqa: E402
from gibbs_student_t_amd.native import NativeSampler  # noqa: E402

W, H, B = _abi.STAGE_WHITE, _abi.STAGE_HYPER, _abi.STAGE_B
TZA, DF = _abi.STAGE_THETA | _abi.STAGE_Z | _abi.STAGE_ALPHA, _abi.STAGE_DF
MASKS = [("all", _abi.STAGE_ALL), ("no toa stages", W | H | B), ("no b draw", W | H | TZA | DF),
         ("white + hyper", W | H), ("hyper only", H), ("white only", W), ("theta only", _abi.STAGE_THETA),
         ("z only", _abi.STAGE_Z), ("alpha only", _abi.STAGE_ALPHA), ("nu only", DF),
         ("nothing", 0)]


def main():
    C = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    S = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    if len(sys.argv) > 3 and sys.argv[3] == "c3":
        out, _ = data.simulate_data(seed=2017, theta=0.05, red_source="red.txt")
        pta = PTA(out)
    else:
        pta = PTA(data.j1713())
    ns = NativeSampler(pta, dict(model="mixture", vary_df=True, theta_prior="beta"), 0)
    ns.alloc(C)
    rng = np.random.default_rng(0)
    lo = np.array([p.pmin for p in pta.params])
    hi = np.array([p.pmax for p in pta.params])
    ns.set_state(x=rng.uniform(lo, hi, size=(C, len(lo))), z=np.ones((C, ns.n)),
                 alpha=np.ones((C, ns.n)), theta=np.full(C, 0.01), nu=np.full(C, 4.0))
    ns.sweep(300, seed=1)                      # burn in: realistic acceptance / redraw rates
    st = ns.get_state()
    res = {}
    for name, mask in MASKS:
        ns.set_state(**{k: st[k] for k in ("x", "b", "z", "alpha", "pout", "theta", "nu")})
        ns.sweep(5, seed=2, mask=mask, sweep0=300)
        ns.sweep(S, seed=2, mask=mask, sweep0=305)
        ns.synchronize()
        res[name] = ns.last_kernel_ms() / S * 1e3
        print(f"{name:16s} {res[name]:8.1f} us/sweep", flush=True)
    a = res["all"]
    print(f"toa stages (theta,z,alpha,nu): {a - res['no toa stages']:.1f} us")
    print(f"b draw (+ T b):               {a - res['no b draw']:.1f} us")
    print(f"white MH:                     {res['white + hyper'] - res['hyper only']:.1f} us")
    print(f"gram + hyper MH:              {res['hyper only'] - res['nothing']:.1f} us")
    print(f"fixed (records, launch):      {res['nothing']:.1f} us")
    for k in ("white only", "theta only", "z only", "alpha only", "nu only"):
        print(f"{k:30s} {res[k] - res['nothing']:.1f} us")


if __name__ == "__main__":
    main()
