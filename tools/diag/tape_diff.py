"""Replay a fixture's tape on two libgst builds and print the first differing record per
key (records are the state at the START of each sweep, so record i + 1 holds sweep i's draws).

    python tools/diag/tape_diff.py LIB_A LIB_B [fixture] [chains]
"""
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
KEYS = ("x", "b", "z", "alpha", "pout", "theta", "nu")


def worker(name, C, out):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch
    from golden_io import load_ref, sweep_state
    from gibbs_student_t_amd.native import NativeSampler, pack_tape
    ref = load_ref(name)
    S = int(ref["niter"])
    s0 = sweep_state(ref, 0)
    ns = NativeSampler(ref["pta"], ref["kw"], 0)
    if os.environ.get("TD_POISON") == "1":
        ns.set_debug(poison=True)
    ns.alloc(C)
    rep = lambda a: np.repeat(np.asarray(a)[None], C, axis=0)  # noqa: E731
    ns.set_state(x=rep(ref["xs"]), b=rep(s0["b"]), z=rep(s0["z"]), alpha=rep(s0["alpha"]),
                 pout=rep(s0["pout"]), theta=np.full(C, s0["theta"]), nu=np.full(C, s0["nu"]))
    rows = pack_tape(ref["tape"], np.arange(S), ns.n, ns.m, ns.stride)
    tape = torch.as_tensor(np.repeat(rows[None], C, axis=0)).to(ns.tdev).contiguous()
    rec = ns.alloc_records(S)
    ns.sweep(S, records=rec, tape=tape)
    fin = ns.get_state()
    np.savez(out, **{f"rec_{k}": v.cpu().numpy() for k, v in rec.items()},
             **{f"fin_{k}": v for k, v in fin.items()})


def main():
    if sys.argv[1] == "--worker":
        worker(sys.argv[2], int(sys.argv[3]), sys.argv[4])
        return 0
    a, b = sys.argv[1], sys.argv[2]
    name = sys.argv[3] if len(sys.argv) > 3 else "mid_beta_fixed"
    C = int(sys.argv[4]) if len(sys.argv) > 4 else 1
    with tempfile.TemporaryDirectory() as td:
        outs = []
        for side, lib in enumerate((a, b)):
            out = os.path.join(td, f"{side}_" + os.path.basename(lib) + ".npz")
            env = dict(os.environ, GST_LIB=os.path.abspath(lib))
            # TD_POISON_B=1: the second run overwrites the chain's LDS and parked TM factor
            # with NaN at the start of every sweep (gst_set_debug)
            env["TD_POISON"] = "1" if (side == 1 and os.environ.get("TD_POISON_B") == "1") else "0"
            subprocess.run([sys.executable, os.path.abspath(__file__), "--worker", name, str(C),
                            out], env=env, check=True)
            outs.append(np.load(out))
    for k in outs[0].files:
        u, v = outs[0][k], outs[1][k]
        if np.array_equal(u, v):
            print(f"{k}: identical")
            continue
        d = np.abs(u - v)
        if k.startswith("rec_"):
            per = d.reshape(d.shape[0], d.shape[1], -1).max(axis=(0, 2))
            first = int(np.argmax(per > 0))
            print(f"{k}: first differing record {first}, max |diff| per record "
                  f"{np.array2string(per, precision=2)}")
            if u.ndim == 3:
                idx = np.nonzero(d[0, first] > 0)[0]
                print(f"   record {first} chain 0: {len(idx)} entries differ, at {idx[:20]}; "
                      f"A {u[0, first, idx[:5]]} B {v[0, first, idx[:5]]}")
        else:
            print(f"{k}: max |diff| {d.max():.3e}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
