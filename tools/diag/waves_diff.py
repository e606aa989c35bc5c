"""Where do the one-wave and two-wave kernels first differ (tests/test_gpu_waves.py setup)?
    python tools/diag/waves_diff.py [fixture]"""
import sys

import numpy as np

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from test_gpu_waves import KEYS, _init, _run  # noqa: E402
import test_gpu_waves  # noqa: E402
from golden_io import load_ref  # noqa: E402
from gibbs_student_t_amd import _abi  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "beta_efac_fixed"
ref = load_ref(name)
import os
C, S = int(os.environ.get("WD_C", 96)), int(os.environ.get("WD_S", 24))
init = _init(ref, C, 5)
one, r1 = _run(ref, C, S, 1, init)
two, r2 = _run(ref, C, S, 2, init)
bad = set()
for k in KEYS:
    d = np.any((r1[k] != r2[k]).reshape(C, S, -1), axis=2)
    for c in np.nonzero(d.any(axis=1))[0]:
        s = int(np.argmax(d[c]))
        bad.add((int(c), s))
        print(f"{k:6s} chain {c}: first differing record at sweep {s}")
for c, s in sorted(bad)[:3]:
    print(f"chain {c} sweep {s - 1} -> {s}: x1 {r1['x'][c, s - 1]} / {r1['x'][c, s]}, x2 {r2['x'][c, s]}")
    print("  b diff", np.max(np.abs(r1['b'][c, s] - r2['b'][c, s])), "alpha", np.max(np.abs(r1['alpha'][c, s] - r2['alpha'][c, s])))
    # replay that sweep stage by stage from the common start state
    st = {k: r1[k][c:c + 1, s - 1].copy() for k in KEYS}
    acc = 0
    for bit, nm in ((1, "white"), (2, "hyper"), (4, "b"), (8, "theta"), (16, "z"), (32, "alpha"), (64, "nu")):
        acc |= bit
        o1, _ = _run(ref, 1, 1, 1, st, mask=acc, sweep0=3 + s - 1)
        o2, _ = _run(ref, 1, 1, 2, st, mask=acc, sweep0=3 + s - 1)
        eq = {k: bool(np.array_equal(o1[k], o2[k])) for k in KEYS}
        print(f"  through {nm:6s}: " + " ".join(f"{k}={'=' if v else 'X'}" for k, v in eq.items()),
              f"max|dz| {np.max(np.abs(o1['z'] - o2['z']))} max|dpout| {np.max(np.abs(o1['pout'] - o2['pout'])):.3e}")
