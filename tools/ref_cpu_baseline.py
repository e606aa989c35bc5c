"""CPU baseline of the REFERENCE sampler itself, timed in this container.

The reference ``gibbs.py`` (only shim: Python-2 ``map``) never travels to the GPU box, so
``bench.py``'s ``cpu_baseline`` there times the oracle port.  This script times both on the
same host, same workload, side by side: the bench config-2 dataset (``data.j1713()``, the
run_sims 'beta' mixture model), one chain per process, single-threaded BLAS, P processes,
each running S sweeps from its own prior draw (run_sims.py:111).  It reports aggregate
chain-sweeps/s and ESS/s (min over {gamma, log10_A, log10_equad, theta} of the bulk ESS
summed over chains / wall time of the slowest process), with the core count.

    python tools/ref_cpu_baseline.py [processes] [sweeps]   -> profiles/cpu_reference_container.json
"""
from __future__ import annotations

import builtins
import json
import os
import platform
import subprocess
import sys
import tempfile
import time
import warnings

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
CFG = dict(model="mixture", vary_df=True, theta_prior="beta")   # run_sims.py:98-99
BURN = 200


def worker(kind: str, sweeps: int, seed: int, path: str):
    sys.dont_write_bytecode = True
    sys.path.insert(0, ROOT)
    warnings.filterwarnings("ignore")
    from gibbs_student_t_amd import data
    from gibbs_student_t_amd.model import PTA
    pta = PTA(data.j1713())
    np.random.seed(seed)
    xs = pta.sample_params()
    if kind == "reference":
        sys.path.insert(0, "/root/reference")
        import gibbs as refgibbs  # the reference, gibbs.py:9-385
        refgibbs.map = lambda f, *a: list(builtins.map(f, *a))
        g = refgibbs.Gibbs(pta, **CFG)
        t0 = time.perf_counter()
        g.sample(xs, niter=sweeps)
        dt = time.perf_counter() - t0
        x, th = g.chain, g.thetachain
    else:
        from oracle.gibbs_oracle import LegacyNumpyVariates, Oracle, OutlierModel, initial_state
        orc = Oracle(pta, OutlierModel(**CFG))
        st = initial_state(pta, orc.cfg)
        src = LegacyNumpyVariates()
        x = np.zeros((sweeps, len(xs)))
        th = np.zeros(sweeps)
        t0 = time.perf_counter()
        for i in range(sweeps):
            x[i], th[i] = xs, st.theta        # state at the start of the sweep (gibbs.py:355)
            xs = orc.sweep(st, xs, src)
        dt = time.perf_counter() - t0
    np.savez(path, x=x, theta=th, seconds=dt, names=np.array([p.name for p in pta.params]))


def run(kind: str, procs: int, sweeps: int):
    sys.path.insert(0, ROOT)
    from gibbs_student_t_amd import diag
    env = dict(os.environ, OPENBLAS_NUM_THREADS="1", OMP_NUM_THREADS="1", MKL_NUM_THREADS="1")
    tmp = tempfile.mkdtemp(prefix="gst_cpu_")
    paths = [os.path.join(tmp, f"{kind}_{i}.npz") for i in range(procs)]
    t0 = time.perf_counter()
    ps = [subprocess.Popen([sys.executable, os.path.abspath(__file__), "--worker", kind,
                            str(sweeps), str(4242 + i), paths[i]], env=env)
          for i in range(procs)]
    for p in ps:
        assert p.wait() == 0, f"{kind} worker failed"
    wall = time.perf_counter() - t0
    parts = [np.load(p) for p in paths]
    secs = [float(p["seconds"]) for p in parts]
    xs = np.stack([p["x"][BURN:] for p in parts])
    th = np.stack([p["theta"][BURN:] for p in parts])
    names = [str(s).split("_", 1)[1] for s in parts[0]["names"]]
    ess = {nm: float(diag.bulk_ess(xs[:, :, j])) for j, nm in enumerate(names)}
    ess["theta"] = float(diag.bulk_ess(th))
    for p in paths:
        os.remove(p)
    os.rmdir(tmp)
    slowest = max(secs)
    return {"kind": kind, "processes": procs, "sweeps_per_chain": sweeps, "burn_in": BURN,
            "chain_sweeps_per_s": procs * sweeps / slowest,
            "per_core_sweeps_per_s": float(np.mean([sweeps / s for s in secs])),
            "ess_total": ess, "ess_per_s": min(ess.values()) / slowest,
            "sampling_seconds_max": slowest, "wall_incl_startup_s": wall}


def main():
    if sys.argv[1:2] == ["--worker"]:
        worker(sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), sys.argv[5])
        return
    procs = int(sys.argv[1]) if len(sys.argv) > 1 else (os.cpu_count() or 8)
    sweeps = int(sys.argv[2]) if len(sys.argv) > 2 else 4000
    out = {"host": {"cpu": platform.processor() or platform.machine(),
                    "cores_used": procs, "blas_threads_per_process": 1},
           "workload": "bench.py config 2 dataset (data.j1713(): 130 J1713+0747 epochs, m=74), "
                       "run_sims 'beta' mixture model, one chain per process from a prior draw",
           "runs": [run("reference", procs, sweeps), run("port", procs, sweeps)]}
    r, o = out["runs"]
    out["port_over_reference"] = o["per_core_sweeps_per_s"] / r["per_core_sweeps_per_s"]
    dst = os.path.join(ROOT, "profiles", "cpu_reference_container.json")
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
