"""Where do the one-wave and two-wave kernels first differ (tests/test_gpu_waves.py setup)?
    python tools/diag/waves_diff.py [fixture]

For each differing chain c, the sweep before its first differing record is replayed
stage by stage in fresh one-chain launches of both kernels, from chain c's recorded state
and with chain c's own Philox stream (chain0 = c: a launch's chain j draws from global
chain chain0 + j).  If every stage of the replay agrees, the divergence needs state that
the records do not carry (LDS / register contents from earlier sweeps of the launch)."""
import os
import sys

import numpy as np

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from test_gpu_waves import KEYS, _init, _run  # noqa: E402
from golden_io import load_ref  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "beta_efac_fixed"
ref = load_ref(name)
C, S = int(os.environ.get("WD_C", 96)), int(os.environ.get("WD_S", 24))
SWEEP0, SEED = 3, 7
init = _init(ref, C, 5)
one, r1 = _run(ref, C, S, 1, init, seed=SEED, sweep0=SWEEP0)
two, r2 = _run(ref, C, S, 2, init, seed=SEED, sweep0=SWEEP0)
first = {}
for k in KEYS:
    d = np.any((r1[k] != r2[k]).reshape(C, S, -1), axis=2)
    for c in np.nonzero(d.any(axis=1))[0]:
        s = int(np.argmax(d[c]))
        first[int(c)] = min(first.get(int(c), S), s)
        print(f"{k:6s} chain {c}: first differing record {s}")
print(f"{len(first)} of {C} chains differ")
for c, s in sorted(first.items())[:4]:
    if s == 0:
        continue
    print(f"chain {c}: records {s - 1} equal, record {s} differs; replaying sweep {s - 1}")
    for k in KEYS:
        print(f"  record {s} {k}: max|one - two| {np.max(np.abs(r1[k][c, s] - r2[k][c, s])):.3e}")
    st = {k: r1[k][c:c + 1, s - 1].copy() for k in KEYS}
    acc = 0
    for bit, nm in ((1, "white"), (2, "hyper"), (4, "b"), (8, "theta"), (16, "z"), (32, "alpha"),
                    (64, "nu")):
        acc |= bit
        o1, _ = _run(ref, 1, 1, 1, st, mask=acc, seed=SEED, sweep0=SWEEP0 + s - 1, chain0=c)
        o2, _ = _run(ref, 1, 1, 2, st, mask=acc, seed=SEED, sweep0=SWEEP0 + s - 1, chain0=c)
        eq = {k: bool(np.array_equal(o1[k], o2[k])) for k in KEYS}
        # the full-sweep replay must reproduce the long launch's record s on each side
        tail = ""
        if acc == 0x7F:
            rep1 = all(np.array_equal(o1[k][0], r1[k][c, s]) for k in KEYS)
            rep2 = all(np.array_equal(o2[k][0], r2[k][c, s]) for k in KEYS)
            tail = f" | replay == long launch: one-wave {rep1}, two-wave {rep2}"
        print(f"  through {nm:6s}: " + " ".join(f"{k}={'=' if v else 'X'}" for k, v in eq.items())
              + tail)
