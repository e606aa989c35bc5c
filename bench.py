"""Benchmark: aggregate Gibbs sweeps/s (+ ESS/s) on J1713+0747, batched chains per GPU.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--chains C] [--config 2|3|4]

A *step* is one Gibbs sweep (gibbs.py:354-380) of every chain on every rank.  Each rank
owns C chains (weak scaling, default 1024 = BASELINE config 2 per GPU) of the run_sims.py
'beta' outlier-mixture model (run_sims.py:98-99) on J1713+0747's 130 TOAs; the timed region
is exactly K sweeps in one persistent launch, recording every sweep's full state (chain,
bchain, zchain, alphachain, poutchain, thetachain, dfchain) to HBM as the reference records
every sweep.  For N > 1 the driver starts one process per GPU with torch.distributed.run;
chains never communicate while sampling, the only collective is the final summary
all-reduce (RCCL).  Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Gibbs sweeps/sec (node aggregate) + ESS/sec, J1713+0747, 1/2/4/8 GPU"
FP64_PEAK_TFLOPS = 78.6      # MI355X fp64 matrix (= vector) dense peak, AMD spec
HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md: 8.0 TB/s spec
CFG = dict(model="mixture", vary_df=True, theta_prior="beta")   # run_sims.py:98-99


def algorithmic_flops(n: int, m: int) -> float:
    """Fixed work per chain-sweep: Gram of [T|r], 12 Cholesky (11 MH + 1
    draw), 12 pairs of triangular solves, one T b."""
    return n * (m + 1) * (m + 2) + 12 * m ** 3 / 3 + 12 * 4 * m ** 2 + 2 * n * m


def toa_pass_bytes(n: int) -> float:
    """Per-TOA pass HBM bytes per chain-sweep: 8 n (6 + 2*21)."""
    return 8.0 * n * (6 + 2 * 21)


# ------------------------------------------------------------------------------------------
# CPU baseline: the oracle (a faithful port of gibbs.py, bit-exact to the reference on the
# same MT19937 stream) timed on host cores, one chain per single-threaded process.
# ------------------------------------------------------------------------------------------
def _cpu_worker(seconds: float, seed: int):
    import warnings

    from gibbs_student_t_amd import data
    from gibbs_student_t_amd.model import PTA
    from oracle.gibbs_oracle import (LegacyNumpyVariates, Oracle, OutlierModel,
                                     initial_state)
    warnings.simplefilter("ignore")
    pta = PTA(data.j1713())
    orc = Oracle(pta, OutlierModel(**CFG))
    np.random.seed(seed)
    x = pta.sample_params()
    st = initial_state(pta, orc.cfg)
    src = LegacyNumpyVariates()
    for _ in range(3):
        x = orc.sweep(st, x, src)
    t0 = time.perf_counter()
    k = 0
    while time.perf_counter() - t0 < seconds:
        x = orc.sweep(st, x, src)
        k += 1
    print(json.dumps({"sweeps": k, "seconds": time.perf_counter() - t0}))


def cpu_baseline(seconds: float, cores: int):
    env = dict(os.environ, OPENBLAS_NUM_THREADS="1", OMP_NUM_THREADS="1",
               MKL_NUM_THREADS="1", HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="")
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__), "--cpu-worker",
                               str(seconds), str(1000 + i)], env=env, stdout=subprocess.PIPE,
                              stderr=subprocess.DEVNULL, text=True) for i in range(cores)]
    tot = 0.0
    sweeps = 0
    for p in procs:
        out, _ = p.communicate(timeout=seconds * 10 + 120)
        r = json.loads(out.strip().splitlines()[-1])
        tot += r["sweeps"] / r["seconds"]
        sweeps += r["sweeps"]
    return {"value": tot, "unit": "chain-sweeps/s", "cores": cores, "kind": "port",
            "sample": f"{cores} single-thread processes x {seconds:.0f} s of the oracle "
                      f"(oracle/gibbs_oracle.py, numpy legacy RNG, bit-exact to gibbs.py), "
                      f"one J1713 mixture chain each, {sweeps} sweeps total"}


# ------------------------------------------------------------------------------------------
def initial_state(pta, C: int, chain0: int):
    """Prior draws per global chain id (run_sims.py:111) and the gibbs.py:29-51 latents."""
    n, m = pta.T.shape
    lo = np.array([p.pmin for p in pta.params])
    hi = np.array([p.pmax for p in pta.params])
    x = np.stack([np.random.default_rng([7, chain0 + c]).uniform(lo, hi) for c in range(C)])
    return dict(x=x, b=np.zeros((C, m)), z=np.ones((C, n)), alpha=np.ones((C, n)),
                pout=np.zeros((C, n)), theta=np.full(C, 0.01), nu=np.full(C, 4.0))


def workload(config: int, rank: int, world: int, chains: int | None):
    """BASELINE.json configs as (datasets, cfgs, chain->dataset, initial state, description).

    2: J1713+0747 epochs, 1024 chains per GPU (the headline, default);
    3: simulate_data.py pulsar, 5% outliers, red.txt red noise, 512 chains per GPU
       (4096 over 8 GPUs);
    4: run_sims.py grid, 256 datasets (3 outlier fractions x {Gaussian, Student-t nu=4}
       white noise x outlier/no_outlier twins x 5 outlier models) x 64 chains, 32
       datasets per GPU.
    All weak scaling: the per-GPU work is fixed as the GPU count grows.
    """
    from gibbs_student_t_amd import data
    from gibbs_student_t_amd import run_sims
    from gibbs_student_t_amd.model import PTA
    if config in (2, 3):
        if config == 2:
            pta = PTA(data.j1713())
            C = chains or 1024
            desc = ("J1713+0747 Student-t/outlier-mixture Gibbs sampler (run_sims 'beta' "
                    "model), fp64")
            dat = ("synthetic residuals at the 130 real J1713+0747 TOA epochs (white + "
                   "power-law red + 5% outliers, seeded); chains start from prior draws")
        else:
            out, _ = data.simulate_data(seed=2017, theta=0.05, red_source="red.txt")
            pta = PTA(out)
            C = chains or 512
            desc = ("simulate_data.py pulsar (J1713+0747 epochs, log-normal errors, red.txt "
                    "red noise, 5% outliers), run_sims 'beta' model, fp64")
            dat = ("simulate_data.py restatement: log-normal error bars, the reference's "
                   "red.txt realisation, Bernoulli(0.05) outliers with sigma_out = 1 us")
        c0 = rank * C
        return dict(ptas=[pta], cfgs=[CFG], ds=np.zeros(C, np.int32),
                    init=initial_state(pta, C, c0), chain0=c0, C=C, desc=desc, data=dat,
                    per=C)
    if config == 4:
        per_entry = chains or 64
        grid = run_sims.build_grid(thetas=(0.05, 0.1, 0.15), realisations=5,
                                   dofs=(None, 4.0))[:256]
        per_rank = 256 // 8 if world <= 8 else max(1, 256 // world)
        e0 = rank * per_rank
        mine = grid[e0:e0 + per_rank]
        nst = max(e.pta.n for e in mine)
        parts = [run_sims.initial_state(e, per_entry, (e0 + i) * per_entry, 7, nst)
                 for i, e in enumerate(mine)]
        init = {k: np.concatenate([p_[k] for p_ in parts]) for k in parts[0]}
        C = len(mine) * per_entry
        return dict(ptas=[e.pta for e in mine], cfgs=[e.cfg for e in mine],
                    ds=np.repeat(np.arange(len(mine)), per_entry).astype(np.int32), init=init,
                    chain0=e0 * per_entry, C=C, per=per_entry,
                    desc=("run_sims.py grid: 256 simulated datasets (theta 0.05/0.1/0.15, "
                          "Gaussian and Student-t nu=4 white noise, outlier + no_outlier "
                          "twins, 5 outlier models) x 64 chains, 32 datasets per GPU, fp64"),
                    data="simulate_data.py restatement per dataset (seeded), ragged n")
    if config == 5:
        psr = data.scaled_synthetic(n=100_000, components=60, ntm=300, seed=5)
        pta = PTA(psr, components=60)
        C = chains or 512
        c0 = rank * C
        return dict(ptas=[pta], cfgs=[CFG], ds=np.zeros(C, np.int32),
                    init=initial_state(pta, C, c0), chain0=c0, C=C, per=C,
                    desc=("scaled synthetic pulsar: 100k TOAs over 10 yr, 60 red-noise "
                          "components (120 Fourier columns) + 300 timing/DMX columns (m=420), "
                          "run_sims 'beta' model, 512 chains per GPU, fp64, large-model path"),
                    data=("data.scaled_synthetic: log-normal error bars, power-law red noise, "
                          "5% outliers, random 300-column timing/DMX design matrix projected "
                          "out; records x, b, theta, nu every sweep (per-TOA chains not "
                          "recorded: 1.2 GB per sweep)"))
    raise SystemExit(f"unknown --config {config}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=300)
    ap.add_argument("--config", type=int, default=2, choices=(2, 3, 4, 5),
                    help="BASELINE.json config (2 = headline J1713+0747, 1024 chains/GPU)")
    ap.add_argument("--chains", type=int, default=None,
                    help="chains per GPU (config 4: per dataset)")
    ap.add_argument("--seed", type=int, default=20171713)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-worker", nargs=2, default=None)
    args = ap.parse_args()
    if args.cpu_worker:
        _cpu_worker(float(args.cpu_worker[0]), int(args.cpu_worker[1]))
        return

    from gibbs_student_t_amd import dist
    rank, local, world = dist.env_rank()
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cores = max(1, min(16, os.cpu_count() or 1))
        cpu = cpu_baseline(args.cpu_seconds, cores)      # before the GPU is touched

    import torch
    from gibbs_student_t_amd import diag
    from gibbs_student_t_amd.native import NativeSampler

    rank, local, world = dist.init()
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    wl = workload(args.config, rank, world, args.chains)
    C, K, W = wl["C"], args.steps, args.warmup
    c0 = wl["chain0"]
    ns = NativeSampler(wl["ptas"], wl["cfgs"], local)
    ns.alloc(C, dataset=wl["ds"])
    ns.set_state(**wl["init"])
    if W > 0:
        ns.sweep(W, seed=args.seed, sweep0=0, chain0=c0)
    large = ns.path == "large"
    rec = ns.alloc_records(K, keys=("x", "b", "theta", "nu") if large else
                           ("x", "b", "z", "alpha", "pout", "theta", "nu"))
    if large:
        ns.set_timing(True)
    torch.cuda.synchronize(dev)
    dist.barrier(dev)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ns.sweep(K, records=rec, seed=args.seed, sweep0=W, chain0=c0)
    torch.cuda.synchronize(dev)
    dist.barrier(dev)
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    kernel_ms = ns.last_kernel_ms()
    ktimes = ns.kernel_times() if large else None
    status = ns.get_state()["status"]

    # ESS per dataset (its chains share one posterior), summed over datasets and ranks
    xs = rec["x"].cpu().numpy()
    th = rec["theta"].cpu().numpy()
    names = [p.name.split("_", 1)[1] for p in wl["ptas"][0].params]
    keys = names + ["theta"]
    ess = {k: 0.0 for k in keys}
    rhat = {k: 0.0 for k in keys}
    for d in range(len(wl["ptas"])):
        sel = wl["ds"] == d
        series = {nm: xs[sel, :, j] for j, nm in enumerate(names)}
        series["theta"] = th[sel]
        for k, v in series.items():
            if k == "theta" and wl["cfgs"][d]["model"] not in ("mixture", "vvh17"):
                continue            # theta is never updated: no ESS to speak of
            e = diag.bulk_ess(v)
            ess[k] += e if np.isfinite(e) else 0.0
            r = diag.split_rhat(v)
            rhat[k] = max(rhat[k], r if np.isfinite(r) else 0.0)
    s_vec = np.array([ess[k] for k in keys] + [float((status != 0).sum())])
    m_vec = np.array([elapsed, kernel_ms] + [rhat[k] for k in keys])
    s_vec, m_vec = dist.reduce_summary(s_vec, m_vec, dev)
    elapsed, kernel_ms = float(m_vec[0]), float(m_vec[1])
    ess_tot = dict(zip(keys, s_vec[:len(keys)]))
    rhat_max = dict(zip(keys, m_vec[2:]))

    if rank == 0:
        total = C * world * K
        value = total / elapsed
        n_mean = float(np.mean([p_.T.shape[0] for p_ in wl["ptas"]]))
        n, m = wl["ptas"][0].T.shape
        n_eff = n if args.config != 4 else n_mean
        flops = algorithmic_flops(n_eff, m) * C * K
        achieved = flops / (kernel_ms * 1e-3) / 1e12
        stages = None
        toa_ms = kernel_ms
        if ktimes:
            # dominant kernel = the Gram; its algorithmic flops per launch are the
            # n (m+1) (m+2) term of the fixed formula x chains (one launch per sweep)
            g_ms, g_n = ktimes["gram"]
            gram_flop = n_eff * (m + 1) * (m + 2) * C
            achieved = gram_flop / (g_ms / g_n * 1e-3) / 1e12
            stages = {k: {"ms_per_sweep": v[0] / max(1, K), "launches": v[1]}
                      for k, v in ktimes.items()}
            # per-TOA pass (white MH rescans + theta/z/alpha/nu) over its own kernels' time
            toa_ms = ktimes["white"][0] + ktimes["toa"][0]
        traffic = None
        pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        if os.path.exists(pmc) and args.config == 2:
            try:
                pj = json.load(open(pmc))
                traffic = pj["hbm_bytes_per_chain_sweep"] * C * K
            except Exception:
                traffic = None
        pmc5 = os.path.join(ROOT, "profiles", "pmc_config5.json")
        if large and args.config == 5 and os.path.exists(pmc5):
            try:   # HBM bytes per Gram launch (PMC passes of tools/run_large.py, same shape)
                g = json.load(open(pmc5))["kernels"]["lg_gram"]
                traffic = g["hbm_read_bytes"] + g["hbm_write_bytes"]
            except Exception:
                traffic = None
        pos = [v for v in ess_tot.values() if v > 0]
        min_ess = float(min(pos)) if pos else None
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "chain-sweeps/s",
            "n_gpus": world,
            "steps": K,
            "warmup": W,
            "ms_per_step": elapsed / K * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": wl["data"],
            "config": {"workload": wl["desc"], "baseline_config": args.config,
                       "chains_per_gpu": C, "chains_total": C * world, "n_toa": n,
                       "basis_cols": m, "datasets_per_gpu": len(wl["ptas"]),
                       "record_every": 1,
                       "parallelism": f"independent chains sharded over {world} GPU(s); "
                                      "RCCL only for the final summary all-reduce"},
            "ess_per_sec": (min_ess / elapsed) if min_ess else None,
            "ess_total": {k: float(v) for k, v in ess_tot.items()},
            "rhat_max": {k: float(v) for k, v in rhat_max.items()},
            "chains_with_status": int(s_vec[-1]),
            "kernel_ms": kernel_ms,
            "roofline": {"bound": "mfma", "achieved": achieved, "peak": FP64_PEAK_TFLOPS,
                         "unit": "TFLOP/s", "frac": achieved / FP64_PEAK_TFLOPS,
                         "traffic": traffic,
                         "kernel": "lg_gram (per-launch HIP events)" if large else
                                   "gst_sweep_kernel (persistent, whole launch)",
                         "algorithmic_flop_per_chain_sweep": algorithmic_flops(n_eff, m),
                         "toa_pass_GBps": toa_pass_bytes(n_eff) * C * K / (toa_ms * 1e-3) / 1e9,
                         "toa_pass_hbm_frac": toa_pass_bytes(n_eff) * C * K / (toa_ms * 1e-3)
                         / 1e9 / HBM_PEAK_GBS},
            "cpu_baseline": cpu,
        }
        if stages:
            out["stages"] = stages
        print(json.dumps(out), flush=True)
    ns.close()
    dist.finalize()


if __name__ == "__main__":
    main()
