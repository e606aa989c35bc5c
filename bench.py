"""Benchmark: aggregate Gibbs sweeps/s (+ ESS/s) on J1713+0747, batched chains per GPU.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--chains C] [--config 2|3|4|5]

A *step* is one Gibbs sweep (gibbs.py:354-380) of every chain on every rank.  Each rank owns
C chains (weak scaling; default 2048 per GPU = two chains per SIMD, the "1024+ batched
chains" of the BASELINE metric) of the run_sims.py 'beta' outlier-mixture model (run_sims.py:98-99) on
J1713+0747's 130 TOAs.  The timed region is exactly K sweeps in one persistent launch,
recording every sweep's full state (chain, bchain, zchain, alphachain, poutchain,
thetachain, dfchain) to HBM as the reference records every sweep.

Multi-GPU: one process per GPU.  Under torch.distributed.run the ranks come from the
environment; launched plainly with ``--gpus N > 1`` this script is the launcher: it starts
N rank processes itself (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, 127.0.0.1) before
anything touches a GPU and relays rank 0's JSON line.  Chains never communicate while
sampling; the collectives are the final all-gather of every chain's post-burn-in draws
(global split-R-hat and bulk-ESS over ALL chains) and a max-reduce of the timings.

Order of a run: W warmup sweeps, the timed region (K sweeps), then ``--ess-burn`` burn-in
sweeps (untimed, discarded) and the ESS window.  The burn-in runs AFTER the timed region:
MI355X lowers its shader clock after ~1 s of full load (2.37 -> 2.06 GHz, recovering over
~20 ms of further work; tools/diag/after_burn.py), so a short timed launch right after a
long burn-in launch measures the power manager, not the kernel.  ESS/s has its own window,
independent of --steps: ``--ess-window`` sweeps after the burn-in whose sampled parameters
and theta are recorded every ``--ess-thin``-th sweep, timed on their own; ESS/s = min over
quantities of the bulk-ESS summed over datasets / window seconds, reported only when every
global R-hat is <= 1.01 (else null, with the reason).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
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
RHAT_OK = 1.01
CONFIG4_DATASETS = 256


def algorithmic_flops(n: float, m: int) -> float:
    """Fixed work per chain-sweep: Gram of [T|r], 12 Cholesky (11 MH + 1
    draw), 12 pairs of triangular solves, one T b."""
    return n * (m + 1) * (m + 2) + 12 * m ** 3 / 3 + 12 * 4 * m ** 2 + 2 * n * m


def executed_flops(n: float, nf: int, ntm: int, m: int) -> dict:
    """Flops the Schur-complement algorithm actually performs per chain-sweep:
    the Gram once, the timing-model columns eliminated once, the 11 hyper likelihoods each
    factor only the (nf + 1)-row Fourier block (+ augmented row), the b draw's two solves
    and T b.  Reported next to the fixed formula (SURVEY.md 8d asks for both)."""
    M = ntm + nf + 1                      # system rows incl. the augmented residual row
    gram = n * (m + 1) * (m + 2)
    tm = sum((M - 1 - k) * (M - k) for k in range(ntm))
    hyper = 11 * sum((nf - k) * (nf + 1 - k) for k in range(nf))
    solves = 4 * m * m
    tb = 2 * n * m
    return {"gram": gram, "tm_elim": tm, "hyper_chol": hyper, "b_solves": solves, "tb": tb,
            "total": gram + tm + hyper + solves + tb}


def persistent_shape(nf: int, ntm: int):
    """(MT, K0, RA) of the persistent kernel instance a model runs in (gst.hip kShapes)."""
    for MT, K0, RA in ((8, 2, 56), (10, 2, 76), (10, 3, 76)):
        if 8 * K0 >= max(ntm, 1) and RA - 8 * K0 >= nf:
            return MT, K0, RA
    return None


def gram_path_flops(n: int, nf: int, ntm: int, ncls: int, nflag: float) -> dict:
    """Lane flops one chain-Gram executes on each persistent-kernel path (include/gst.h
    gst_gram_counts).  The instance pads the system to 8 MT rows.
      mfma:     the lower 16x16 tiles of the padded augmented system, ceil(n / 4) k-steps of
                v_mfma_f64_16x16x4 (2 * 16 * 16 * 4 flops each) -- on the MFMA pipe;
      low_rank: per class one FMA per lane per 8x8-cyclic slot (the class Grams), per flagged
                TOA MT row-scaling multiplies + one FMA per slot (its rank-1 update) -- on
                the VALU.
    Executed (padded) work, not SURVEY.md 8d's algorithmic n (m+1)(m+2)."""
    sh = persistent_shape(nf, ntm)
    if sh is None:
        return {"mfma": float("nan"), "low_rank": float("nan")}
    MT = sh[0]
    NT = (sh[2] + 1 + 15) // 16
    nsl = MT * (MT + 1) // 2
    return {"mfma": NT * (NT + 1) / 2 * ((n + 3) // 4) * 2 * 16 * 16 * 4,
            "low_rank": 64.0 * (ncls * 2 * nsl + nflag * (2 * nsl + MT))}


def pmc_mfma(pf: str | None):
    """MFMA work the committed PMC pass of the same command counted (rocprofv3 --pmc
    SQ_INSTS_VALU_MFMA_MOPS_F64 (units of 512 flops) and SQ_VALU_MFMA_BUSY_CYCLES), per
    chain-sweep, next to the fp64 VALU FMA count: what the Gram executes on which pipe."""
    if not pf or not os.path.exists(pf):
        return None
    try:
        pj = json.load(open(pf))
        cs = float(pj["chains"]) * float(pj["sweeps"])
        return {"source": os.path.relpath(pf, ROOT) + " (rocprofv3 --pmc pass of bench.py, "
                          "not this run)",
                "mfma_flop_per_chain_sweep": pj["SQ_INSTS_VALU_MFMA_MOPS_F64"] * 512.0 / cs,
                "mfma_busy_cycles_per_chain_sweep": pj["SQ_VALU_MFMA_BUSY_CYCLES"] / cs,
                "valu_fma_f64_insts_per_chain_sweep": pj["SQ_INSTS_VALU_FMA_F64"] / cs,
                "valu_insts_per_chain_sweep": pj["SQ_INSTS_VALU"] / cs}
    except (KeyError, ValueError, OSError):
        return None


def stage_costs(ns, S: int, seed: int, sweep0: int, chain0: int) -> dict:
    """Per-sweep kernel time (ms, HIP events) of stage-masked persistent launches: nothing
    (launch + state load/store), the per-TOA pass (white MH + theta, z, alpha, nu), the Gram
    with the timing-model elimination only (GST_STAGE_GRAM), and the whole red-noise block
    (Gram + the 11 likelihood factorisations).  Run after the ESS window: they move the
    chains, which no longer matters then."""
    from gibbs_student_t_amd import _abi
    toa = _abi.STAGE_WHITE | _abi.STAGE_THETA | _abi.STAGE_Z | _abi.STAGE_ALPHA | _abi.STAGE_DF
    out = {}
    # a full-mask launch first: after host-side work the GPU is ramping its clock back up
    # from idle, which would be charged to whichever stage launch came first
    ns.sweep(S, seed=seed, sweep0=sweep0, chain0=chain0)
    for name, mask in (("fixed", 0), ("toa_pass", toa), ("gram", _abi.STAGE_GRAM),
                       ("hyper", _abi.STAGE_HYPER)):
        t = []
        ns.gram_counts(reset=True)
        for rep in range(2):        # the faster of two launches of each
            ns.sweep(S, seed=seed, sweep0=sweep0, chain0=chain0, mask=mask)
            ns.synchronize()
            t.append(ns.last_kernel_ms() / S)
        out[name] = min(t)
        out[name + "_gram_paths"] = ns.gram_counts(reset=True)
    return out


def noise_classes(pta) -> int:
    """Noise classes of a dataset as gst_model_set forms them (equal error bar and backend;
    0 past 8: the per-TOA white likelihood and the MFMA Gram)."""
    err = np.asarray(pta._toaerrs)
    keys = set(zip((err * err).tolist(), np.asarray(pta.bidx).tolist()))
    return len(keys) if len(keys) <= 8 else 0


def toa_pass_bytes(n: float) -> float:
    """Per-TOA pass HBM bytes per chain-sweep: 8 n (6 + 2*21)."""
    return 8.0 * n * (6 + 2 * 21)


# ------------------------------------------------------------------------------------------
# workloads (BASELINE.json configs)
# ------------------------------------------------------------------------------------------
def initial_state(pta, C: int, chain0: int):
    """Prior draws per global chain id (run_sims.py:111) and the gibbs.py:29-51 latents."""
    n, m = pta.T.shape
    lo = np.array([p.pmin for p in pta.params])
    hi = np.array([p.pmax for p in pta.params])
    x = np.stack([np.random.default_rng([7, chain0 + c]).uniform(lo, hi) for c in range(C)])
    return dict(x=x, b=np.zeros((C, m)), z=np.ones((C, n)), alpha=np.ones((C, n)),
                pout=np.zeros((C, n)), theta=np.full(C, 0.01), nu=np.full(C, 4.0))


def config_datasets(config: int):
    """(ptas, cfgs) of a config's whole job, in global order (no sharding)."""
    from gibbs_student_t_amd import data, run_sims
    from gibbs_student_t_amd.model import PTA
    if config == 2:
        return [PTA(data.j1713())], [CFG]
    if config == 3:
        out, _ = data.simulate_data(seed=2017, theta=0.05, red_source="red.txt")
        return [PTA(out)], [CFG]
    if config == 4:
        grid = run_sims.build_grid(thetas=(0.05, 0.1, 0.15), realisations=5,
                                   dofs=(None, 4.0))[:CONFIG4_DATASETS]
        return [e.pta for e in grid], [e.cfg for e in grid]
    if config == 5:
        psr = data.scaled_synthetic(n=100_000, components=60, ntm=300, seed=5)
        return [PTA(psr, components=60)], [CFG]
    raise SystemExit(f"unknown --config {config}")


def workload(config: int, rank: int, world: int, chains: int | None):
    """This rank's share of a BASELINE.json config.

    2: J1713+0747 epochs, 2048 chains per GPU (weak scaling; the headline, default: two
       chains per SIMD, the "1024+" of the BASELINE metric; --chains 1024 for one per SIMD);
    3: simulate_data.py pulsar, 5% outliers, red.txt red noise, 512 chains per GPU
       (4096 over 8 GPUs; weak scaling);
    4: run_sims.py grid: 256 datasets (3 outlier fractions x {Gaussian, Student-t nu=4}
       white noise x outlier/no_outlier twins x 5 outlier models) x 64 chains, the
       datasets sharded over the GPUs (strong scaling: 256 / N datasets per GPU);
    5: scaled synthetic, 100k TOAs, m = 420, 512 chains per GPU (large-model path).
    """
    from gibbs_student_t_amd import run_sims
    if config in (2, 3, 5):
        ptas, cfgs = config_datasets(config)
        C = chains or {2: 2048, 3: 512, 5: 512}[config]
        c0 = rank * C
        desc = {
            2: "J1713+0747 Student-t/outlier-mixture Gibbs sampler (run_sims 'beta' model), fp64",
            3: "simulate_data.py pulsar (J1713+0747 epochs, log-normal errors, red.txt red "
               "noise, 5% outliers), run_sims 'beta' model, fp64",
            5: "scaled synthetic pulsar: 100k TOAs over 10 yr, 60 red-noise components (120 "
               "Fourier columns) + 300 timing/DMX columns (m=420), run_sims 'beta' model, "
               "512 chains per GPU, fp64, large-model path"}[config]
        dat = {
            2: "synthetic residuals at the 130 real J1713+0747 TOA epochs (white + power-law "
               "red + 5% outliers, seeded); chains start from prior draws",
            3: "simulate_data.py restatement: log-normal error bars, the reference's red.txt "
               "realisation, Bernoulli(0.05) outliers with sigma_out = 1 us",
            5: "data.scaled_synthetic: log-normal error bars, power-law red noise, 5% "
               "outliers, random 300-column timing/DMX design matrix projected out; records "
               "x, b, theta, nu every sweep (per-TOA chains not recorded: 1.2 GB per sweep)"}[config]
        return dict(ptas=ptas, cfgs=cfgs, ds=np.zeros(C, np.int32),
                    init=initial_state(ptas[0], C, c0), chain0=c0, C=C, desc=desc, data=dat,
                    per=C, dsid=np.zeros(C, np.int64), scaling="weak")
    if config == 4:
        per_entry = chains or 64
        grid = run_sims.build_grid(thetas=(0.05, 0.1, 0.15), realisations=5,
                                   dofs=(None, 4.0))[:CONFIG4_DATASETS]
        if CONFIG4_DATASETS % world:
            raise SystemExit(f"config 4 shards {CONFIG4_DATASETS} datasets: --gpus must "
                             f"divide it")
        per_rank = CONFIG4_DATASETS // world
        e0 = rank * per_rank
        mine = grid[e0:e0 + per_rank]
        nst = max(e.pta.n for e in mine)
        # every entry starts as gibbs.py:29-51 does (vvh17: z = 1, left through the b draw's
        # SVD noise floor as the reference's chains leave it)
        parts = [run_sims.initial_state(e, per_entry, (e0 + i) * per_entry, 7, nst, "reference")
                 for i, e in enumerate(mine)]
        init = {k: np.concatenate([p_[k] for p_ in parts]) for k in parts[0]}
        C = len(mine) * per_entry
        ds = np.repeat(np.arange(len(mine)), per_entry).astype(np.int32)
        return dict(ptas=[e.pta for e in mine], cfgs=[e.cfg for e in mine], ds=ds, init=init,
                    chain0=e0 * per_entry, C=C, per=per_entry, dsid=(e0 + ds).astype(np.int64),
                    groups_all=np.array([e.model for e in grid]),
                    desc=(f"run_sims.py grid: {CONFIG4_DATASETS} simulated datasets (theta "
                          "0.05/0.1/0.15, Gaussian and Student-t nu=4 white noise, outlier + "
                          "no_outlier twins, 5 outlier models) x 64 chains, datasets sharded "
                          "over the GPUs, fp64"),
                    data="simulate_data.py restatement per dataset (seeded), ragged n",
                    scaling="strong")
    raise SystemExit(f"unknown --config {config}")


# ------------------------------------------------------------------------------------------
# CPU baseline: the oracle (a faithful port of gibbs.py, bit-exact to the reference on the
# same MT19937 stream) timed on host cores, one chain per single-threaded process, on the
# same workload as --config.
# ------------------------------------------------------------------------------------------
def _cpu_worker(config: int, seconds: float, seed: int, slot: int, out: str | None = None):
    import warnings

    from oracle.gibbs_oracle import (LegacyNumpyVariates, Oracle, OutlierModel,
                                     initial_state as orc_init)
    warnings.simplefilter("ignore")
    ptas, cfgs = config_datasets(config)
    k = slot % len(ptas)                      # config 4: the processes cycle the grid
    pta, cfg = ptas[k], cfgs[k]
    orc = Oracle(pta, OutlierModel(**cfg))
    np.random.seed(seed)
    x = pta.sample_params()
    st = orc_init(pta, orc.cfg)
    src = LegacyNumpyVariates()
    x = orc.sweep(st, x, src)
    draws = []
    t0 = time.perf_counter()
    k = 0
    while time.perf_counter() - t0 < seconds:
        x = orc.sweep(st, x, src)
        draws.append(list(x) + [float(st.theta)])    # x and theta at the end of the sweep
        k += 1
    secs = time.perf_counter() - t0
    if out:
        np.save(out, np.asarray(draws, dtype=np.float64))
    print(json.dumps({"sweeps": k, "seconds": secs}))


CPU_ESS_BURN_FRAC = 0.2     # the CPU chains' first fifth (from prior draws) is burn-in


def cpu_ess(draws: list, per_chain_s: list, names: list[str]):
    """ESS/s of the CPU chains (config 2 / 3: every process samples the same posterior):
    rank-normalised bulk-ESS and split-R-hat over all chains, each truncated to the
    shortest chain, after dropping the first CPU_ESS_BURN_FRAC; ESS/s = min over the
    sampled parameters and theta of the ESS / the window's wall time (processes run in
    parallel, so the window takes its share of the slowest process's time)."""
    from gibbs_student_t_amd import diag
    S = min(len(d) for d in draws)
    b = int(CPU_ESS_BURN_FRAC * S)
    if S - b < 40:
        return None
    arr = np.stack([d[b:S] for d in draws])              # [chains, window, P + 1]
    ess, rhat = {}, {}
    for j, nm in enumerate(names + ["theta"]):
        e, r = diag.ess_rhat(arr[:, :, j])
        ess[nm], rhat[nm] = float(e), float(r)
    win_s = max(t * (S - b) / len(d) for t, d in zip(per_chain_s, draws))
    pos = [v for v in ess.values() if v > 0 and np.isfinite(v)]
    return {"ess_per_sec": (min(pos) / win_s) if pos else None, "window_sweeps": S - b,
            "window_seconds": win_s, "ess_total": ess, "rhat_max": rhat}


def cpu_baseline(config: int, seconds: float, cores: int):
    import tempfile
    env = dict(os.environ, OPENBLAS_NUM_THREADS="1", OMP_NUM_THREADS="1",
               MKL_NUM_THREADS="1", HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="")
    with tempfile.TemporaryDirectory() as td:
        outs = [os.path.join(td, f"chain{i}.npy") for i in range(cores)]
        procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__), "--cpu-worker",
                                   str(config), str(seconds), str(1000 + i), str(i), outs[i]],
                                  env=env, stdout=subprocess.PIPE, stderr=subprocess.DEVNULL,
                                  text=True)
                 for i in range(cores)]
        tot, sweeps, secs = 0.0, 0, []
        for p in procs:
            out, _ = p.communicate(timeout=seconds * 10 + 300)
            r = json.loads(out.strip().splitlines()[-1])
            tot += r["sweeps"] / r["seconds"]
            sweeps += r["sweeps"]
            secs.append(r["seconds"])
        ess = None
        if config in (2, 3):
            ptas, _ = config_datasets(config)
            names = [p_.name.split("_", 1)[1] for p_ in ptas[0].params]
            ess = cpu_ess([np.load(o) for o in outs], secs, names)
    what = {2: "one J1713 mixture chain each", 3: "one config-3 (red.txt) mixture chain each",
            4: "each a chain of a different run_sims grid dataset/model",
            5: "one 100k-TOA m=420 mixture chain each"}[config]
    return {"value": tot, "unit": "chain-sweeps/s", "cores": cores, "kind": "port",
            "ess_per_sec": ess["ess_per_sec"] if ess else None,
            "ess": ess if ess else ("n/a: the processes sample different grid datasets"
                                    if config == 4 else "n/a: no ESS window at this size"),
            "sample": f"config {config}: {cores} single-thread processes x {seconds:.0f} s of "
                      f"the oracle (oracle/gibbs_oracle.py, numpy legacy RNG, bit-exact to "
                      f"gibbs.py), {what}, {sweeps} sweeps total"}


# ------------------------------------------------------------------------------------------
# launcher: --gpus N without torch.distributed.run -> N rank processes (never touches a GPU)
# ------------------------------------------------------------------------------------------
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n: int, argv: list[str], poll_s: float = 0.2, grace_s: float = 10.0) -> int:
    """Start N rank processes and relay rank 0's output.  Every child is polled: on the
    first non-zero exit the siblings are terminated (SIGTERM, SIGKILL after ``grace_s``)
    and the launcher returns that exit status, instead of leaving the surviving ranks
    blocked in a collective.  Nothing is exec'd: the ranks are plain children."""
    import threading
    port = str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv,
                                      env=env, stdout=subprocess.PIPE if r == 0 else None,
                                      text=True))
    print("bench launcher: rank pids " + " ".join(str(p.pid) for p in procs), file=sys.stderr,
          flush=True)
    out: list[str] = []
    reader = threading.Thread(target=lambda: out.append(procs[0].stdout.read()), daemon=True)
    reader.start()
    failed = 0
    while True:
        rcs = [p.poll() for p in procs]
        bad = [rc for rc in rcs if rc not in (None, 0)]
        if bad:
            failed = abs(bad[0]) or 1
            break
        if all(rc == 0 for rc in rcs):
            break
        time.sleep(poll_s)
    if failed:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        deadline = time.time() + grace_s
        for p in procs:
            try:
                p.wait(timeout=max(0.1, deadline - time.time()))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
        print(f"bench launcher: a rank exited with status {failed}; terminated the others",
              file=sys.stderr, flush=True)
    reader.join(timeout=grace_s)
    sys.stdout.write("".join(out))
    sys.stdout.flush()
    return failed


# ------------------------------------------------------------------------------------------
# CPU stand-in of the sampler (--stub): lets the launcher, the sharding and the global
# diagnostics be tested on a machine without a GPU.  Each chain is an AR(1) series keyed
# by (seed, global chain id, sweep), so draws do not depend on the sharding.
# ------------------------------------------------------------------------------------------
class StubSampler:
    path = "stub"
    RHO = 0.6

    def __init__(self, ptas, cfgs, device=0):
        import torch
        self.P = len(ptas[0].params)
        self.n, self.m = int(max(p.T.shape[0] for p in ptas)), int(ptas[0].T.shape[1])
        self.tdev = torch.device("cpu")

    def alloc(self, C, dataset=None):
        self.C = int(C)
        self.x = np.zeros((self.C, self.P))
        self.theta = np.zeros(self.C)

    def set_state(self, x=None, theta=None, **_):
        if x is not None:
            self.x[:] = x
        if theta is not None:
            self.theta[:] = theta

    def alloc_records(self, nrec, keys=("x",)):
        import torch
        shapes = {"x": (self.P,), "theta": ()}
        return {k: torch.zeros((self.C, nrec) + shapes.get(k, (1,)), dtype=torch.float64)
                for k in keys}

    def sweep(self, nsweeps, records=None, record_every=1, seed=0, sweep0=0, chain0=0, **_):
        import torch
        r = self.RHO
        for it in range(nsweeps):
            for c in range(self.C):
                rng = np.random.default_rng([seed, chain0 + c, sweep0 + it])
                if records is not None and it % record_every == 0:
                    ri = it // record_every
                    if "x" in records:
                        records["x"][c, ri] = torch.from_numpy(self.x[c])
                    if "theta" in records:
                        records["theta"][c, ri] = float(self.theta[c])
                e = rng.standard_normal(self.P + 1)
                self.x[c] = r * self.x[c] + np.sqrt(1 - r * r) * e[:self.P]
                self.theta[c] = r * self.theta[c] + np.sqrt(1 - r * r) * e[self.P]
        self._ms = 1e-3 * nsweeps

    def last_kernel_ms(self):
        return self._ms

    def get_state(self):
        return {"status": np.zeros(self.C, np.int32)}

    def set_timing(self, on):
        pass

    def kernel_times(self):
        return {}

    def close(self):
        pass


# ------------------------------------------------------------------------------------------
def global_diagnostics(draws: np.ndarray, theta: np.ndarray, dsid: np.ndarray,
                       names: list[str], theta_on: np.ndarray, groups=None):
    """Split-R-hat and bulk-ESS over ALL gathered chains.  ``draws`` [C, S, P], ``theta``
    [C, S], ``dsid`` [C] (dataset of each chain: chains of one dataset share a posterior),
    ``theta_on`` [ndatasets] (theta is updated by the dataset's model).  ESS is summed over
    datasets, R-hat maximised over them; with ``groups`` [ndatasets] (e.g. the outlier model
    of each run_sims entry) the same sums / maxima per group are returned too."""
    from gibbs_student_t_amd import diag
    keys = names + ["theta"]
    ess = {k: 0.0 for k in keys}
    rhat = {k: 0.0 for k in keys}
    by = {}
    conv = {}   # per group: ESS over the datasets whose every R-hat <= RHAT_OK, and counts
    for d in np.unique(dsid):
        sel = dsid == d
        series = {nm: draws[sel, :, j] for j, nm in enumerate(names)}
        if theta_on[d]:
            series["theta"] = theta[sel]
        g = by.setdefault(str(groups[d]), ({k: 0.0 for k in keys}, {k: 0.0 for k in keys})) \
            if groups is not None else None
        de = {}
        dr = 0.0
        for k, v in series.items():
            e, r = diag.ess_rhat(v)
            e = e if np.isfinite(e) else 0.0
            r = r if np.isfinite(r) else np.inf
            ess[k] += e
            rhat[k] = max(rhat[k], r)
            de[k] = e
            dr = max(dr, r)
            if g is not None:
                g[0][k] += e
                g[1][k] = max(g[1][k], r)
        if groups is not None:
            cg = conv.setdefault(str(groups[d]), [{k: 0.0 for k in keys}, 0, 0])
            cg[2] += 1
            if dr <= RHAT_OK:
                cg[1] += 1
                for k, e in de.items():
                    cg[0][k] += e
    if groups is None:
        return ess, rhat
    return ess, rhat, by, conv


def ess_rate(ess, rhat, seconds):
    """ESS/s of the slowest-mixing parameter, or (None, reason) when any R-hat > RHAT_OK."""
    bad = {k: v for k, v in rhat.items() if not v <= RHAT_OK and ess.get(k, 0) > 0}
    pos = [v for v in ess.values() if v > 0]
    if bad:
        return None, f"R-hat > {RHAT_OK} after the window's burn-in: {bad}"
    if pos and seconds > 0:
        return float(min(pos)) / seconds, None
    return None, "n/a"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=300)
    ap.add_argument("--config", type=int, default=2, choices=(2, 3, 4, 5),
                    help="BASELINE.json config (2 = headline J1713+0747)")
    ap.add_argument("--chains", type=int, default=None,
                    help="chains per GPU (config 4: per dataset)")
    ap.add_argument("--seed", type=int, default=20171713)
    ap.add_argument("--ess-burn", type=int, default=None,
                    help="extra discarded sweeps before the ESS window (default 3000; "
                         "config 5: no ESS window)")
    ap.add_argument("--ess-window", type=int, default=None,
                    help="sweeps of the ESS window (default 5000; config 5: 0)")
    ap.add_argument("--ess-thin", type=int, default=5,
                    help="record every k-th sweep of the ESS window (default 5)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-stage-costs", action="store_true",
                    help="skip the stage-masked launches (profiling runs: the timed launch "
                         "stays the last sweep launch)")
    ap.add_argument("--stub", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--stub-fail-rank", type=int, default=-1, help=argparse.SUPPRESS)
    ap.add_argument("--cpu-worker", nargs="+", default=None, help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.cpu_worker:
        w = args.cpu_worker
        _cpu_worker(int(w[0]), float(w[1]), int(w[2]), int(w[3]), w[4] if len(w) > 4 else None)
        return 0

    from gibbs_student_t_amd import dist
    rank, local, world = dist.env_rank()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch_ranks(args.gpus, sys.argv[1:])     # before anything touches a GPU
    cpu = None
    if world == 1 and not args.no_cpu_baseline and not args.stub:
        cores = max(1, min(16 if args.config != 5 else 8, os.cpu_count() or 1))
        secs = args.cpu_seconds if args.config != 5 else max(args.cpu_seconds, 20.0)
        cpu = cpu_baseline(args.config, secs, cores)      # before the GPU is touched
    ess_burn = args.ess_burn if args.ess_burn is not None else (0 if args.config == 5 else 3000)
    ess_win = args.ess_window if args.ess_window is not None else (0 if args.config == 5 else 5000)
    thin = max(1, args.ess_thin)
    ess_win = (ess_win // thin) * thin

    import torch
    rank, local, world = dist.init("gloo" if args.stub else None)
    if args.stub and rank == args.stub_fail_rank:
        return 3                       # launcher test: this rank dies, its peers wait in a collective
    if args.stub:
        dev, Sampler = None, StubSampler

        def sync():
            pass
    else:
        from gibbs_student_t_amd.native import NativeSampler as Sampler
        # local % devices: only ever < 1 on a node with fewer GPUs than ranks, i.e. the
        # gloo rehearsal of several ranks on one GPU (dist.init, GST_DIST_BACKEND)
        dev = torch.device("cuda", local % max(1, torch.cuda.device_count()))
        torch.cuda.set_device(dev)

        def sync():
            torch.cuda.synchronize(dev)
    wl = workload(args.config, rank, world, args.chains)
    C, K, W = wl["C"], args.steps, args.warmup
    c0 = wl["chain0"]
    ns = Sampler(wl["ptas"], wl["cfgs"], dev.index if dev is not None else local)
    ns.alloc(C, dataset=wl["ds"])
    ns.set_state(**wl["init"])
    if W > 0:
        ns.sweep(W, seed=args.seed, sweep0=0, chain0=c0)
    burn = ess_burn if ess_win > 0 else 0
    large = ns.path == "large"
    rec = ns.alloc_records(K, keys=("x", "b", "theta", "nu") if large else
                           ("x", "b", "z", "alpha", "pout", "theta", "nu"))
    if large:
        ns.set_timing(True)

    def timed(fn):
        sync()
        dist.barrier(dev)
        sync()
        t0 = time.perf_counter()
        fn()
        sync()
        dist.barrier(dev)
        sync()
        return time.perf_counter() - t0

    # ---- the timed region: exactly K sweeps, every sweep recorded
    if not args.stub:
        ns.gram_counts(reset=True)    # (synchronises: before the timed region's barrier)
    elapsed = timed(lambda: ns.sweep(K, records=rec, seed=args.seed, sweep0=W, chain0=c0))
    kernel_ms = ns.last_kernel_ms()
    ktimes = ns.kernel_times() if large else None
    status = ns.get_state()["status"]
    # which Gram path each chain-sweep of the timed region took, and the flagged TOAs the
    # low-rank path updates (z at the start of each sweep is the z its Gram uses)
    gram_paths = None if args.stub else ns.gram_counts(reset=True)
    zflag = float(rec["z"].sum(dim=-1).mean()) if "z" in rec else None
    del rec
    if large:
        ns.set_timing(False)

    # ---- ESS window: its own burn-in (discarded) and recorded window, timed on its own
    names = [p.name.split("_", 1)[1] for p in wl["ptas"][0].params]
    ess = rhat = by_group = conv_group = None
    stage_ms = None
    win_s = 0.0
    # b draws at the SVD noise floor (status >> 8 counts them, include/gst.h ABI 5): over the
    # ESS window, i.e. at stationarity (the timed region starts 5 sweeps after prior draws)
    floor_win = None
    if ess_win > 0:
        if burn > 0:
            ns.sweep(burn, seed=args.seed, sweep0=W + K, chain0=c0)
        nfl0 = np.asarray(ns.get_state()["status"]) >> 8
        wrec = ns.alloc_records(ess_win // thin, keys=("x", "theta"))
        win_s = timed(lambda: ns.sweep(ess_win, records=wrec, record_every=thin, seed=args.seed,
                                       sweep0=W + K + burn, chain0=c0))
        nflw = (np.asarray(ns.get_state()["status"]) >> 8) - nfl0
        floor_win = np.array([float((nflw > 0).sum()), float(nflw.sum())])
        if not large and not args.stub and not args.no_stage_costs:   # at the working clock
            stage_ms = stage_costs(ns, max(1, min(K, 200)), args.seed, W + K + burn + ess_win,
                                   c0)
        draws = dist.gather_chains(torch.cat([wrec["x"], wrec["theta"][..., None]], dim=2)
                                   .cpu().numpy(), dev)
        dsid = dist.gather_chains(wl["dsid"].astype(np.float64), dev)
        if rank == 0:
            dsid = dsid.astype(np.int64)
            _, allcfgs = config_datasets(args.config) if args.config == 4 else (None, wl["cfgs"])
            theta_on = np.array([c["model"] in ("mixture", "vvh17") for c in allcfgs])
            groups = wl.get("groups_all")
            res = global_diagnostics(draws[..., :-1], draws[..., -1], dsid, names, theta_on,
                                     groups)
            ess, rhat = res[0], res[1]
            by_group = res[2] if groups is not None else None
            conv_group = res[3] if groups is not None else None
        del wrec, draws
    if stage_ms is None and not large and not args.stub and not args.no_stage_costs:
        stage_ms = stage_costs(ns, max(1, min(K, 200)), args.seed, W + K + burn + ess_win, c0)
    shards = dist.gather_chains(np.array([[c0, c0 + C]], dtype=np.float64), dev)
    m_vec = np.array([elapsed, kernel_ms, win_s])
    # status bit 4 (16) is informational: a b draw at the SVD noise floor (include/gst.h),
    # bits 8.. count them; every other flag of bits 0-7 is an error
    s_vec = np.array([float(((status & 0xef) != 0).sum()), float(((status & 16) != 0).sum()),
                      float((status >> 8).sum())] +
                     (list(floor_win) if floor_win is not None else [0.0, 0.0]))
    s_vec, m_vec = dist.reduce_summary(s_vec, m_vec, dev)
    elapsed, kernel_ms, win_s = (float(v) for v in m_vec)

    if rank == 0:
        total = C * world * K
        value = total / elapsed
        n_mean = float(np.mean([p_.T.shape[0] for p_ in wl["ptas"]]))
        pta0 = wl["ptas"][0]
        n, m = pta0.T.shape
        n_eff = n if args.config != 4 else n_mean
        flops = algorithmic_flops(n_eff, m) * C * K
        achieved = flops / (kernel_ms * 1e-3) / 1e12
        exe = executed_flops(n_eff, pta0.nfourier, pta0.ntm, m)
        stages = None
        toa = None
        if ktimes:
            # dominant kernel = the Gram; its algorithmic flops per launch are the
            # n (m+1) (m+2) term of the fixed formula x chains (one launch per sweep)
            g_ms, g_n = ktimes["gram"]
            gram_flop = n_eff * (m + 1) * (m + 2) * C
            achieved = gram_flop / (g_ms / g_n * 1e-3) / 1e12
            stages = {k: {"ms_per_sweep": v[0] / max(1, K), "launches": v[1]}
                      for k, v in ktimes.items()}
            # the per-TOA pass is its own kernels here (white MH rescans + theta/z/alpha/nu),
            # timed per launch by HIP events
            toa_ms = ktimes["white"][0] + ktimes["toa"][0]
            gbs = toa_pass_bytes(n_eff) * C * K / (toa_ms * 1e-3) / 1e9
            toa = {"kernels": "lg_white + lg_toa (HIP events per launch)",
                   "algorithmic_GBps": gbs,
                   "bytes_per_chain_sweep": toa_pass_bytes(n_eff),
                   "what": "SURVEY.md 8d's algorithmic bytes over the kernels' time, not an HBM "
                           "measurement (HBM bytes: the PMC passes in profiles/*_pmc_config5.json)"}
        traffic, traffic_src = None, None
        # HBM bytes per chain-sweep of the persistent kernel, PMC (FETCH_SIZE x 2 +
        # WRITE_SIZE, MI355X_MICROARCH.md gfx950 correction) at 2048 chains: a rocprofv3
        # --pmc pass of this same command, stored under profiles/ -- NOT measured in this
        # run (counters need their own profiler pass); the newest profile is used
        pmc2 = None
        for pf in ("r6_pmc_config2.json", "r5_pmc_config2.json", "r4_pmc_config2.json",
                   "r3_pmc_config2.json"):
            pmc = os.path.join(ROOT, "profiles", pf)
            if os.path.exists(pmc) and args.config == 2 and not args.stub:
                try:
                    pj = json.load(open(pmc))
                    traffic = pj["hbm_bytes_per_chain_sweep"] * C * K
                    pmc2 = pmc
                    traffic_src = (f"profiles/{pf}: rocprofv3 PMC pass of bench.py (not this "
                                   f"run), {pj['hbm_bytes_per_chain_sweep']:.0f} B per "
                                   "chain-sweep x chains x steps")
                    break
                except Exception:
                    traffic = None
        for pf in ("r6_pmc_config5.json", "r5_pmc_config5.json", "r4_pmc_config5.json",
                   "r3_pmc_config5.json"):
            pmc5 = os.path.join(ROOT, "profiles", pf)
            if large and args.config == 5 and os.path.exists(pmc5):
                try:   # HBM bytes per Gram launch (PMC passes of tools/run_large.py, same shape)
                    g = json.load(open(pmc5))["kernels"]["lg_gram"]
                    traffic = g["hbm_read_bytes"] + g["hbm_write_bytes"]
                    traffic_src = f"profiles/{pf}: rocprofv3 PMC passes (not this run), per launch"
                    break
                except Exception:
                    traffic = None
        stage_rep = None
        if stage_ms is not None:
            fx = stage_ms["fixed"]
            t_toa = max(stage_ms["toa_pass"] - fx, 1e-9)
            t_gram = max(stage_ms["gram"] - fx, 1e-9)
            t_hyp = max(stage_ms["hyper"] - fx, 1e-9)
            gbs = toa_pass_bytes(n_eff) * C / (t_toa * 1e-3) / 1e9
            toa = {"kernels": "gst_sweep_kernel, stage-masked launch (white MH + theta/z/alpha/"
                              "nu) minus an empty launch, HIP events, this run",
                   "ms_per_sweep": t_toa, "onchip_algorithmic_GBps": gbs,
                   "bytes_per_chain_sweep": toa_pass_bytes(n_eff),
                   "what": "SURVEY.md 8d's algorithmic bytes over the stage's time; at these "
                           "sizes they are register / L2-resident, so this is NOT an HBM "
                           "rate (the kernel's HBM bytes: roofline.traffic, PMC)"}
            g_alg = n_eff * (m + 1) * (m + 2)
            pf = gram_path_flops(int(n), pta0.nfourier, pta0.ntm, noise_classes(pta0),
                                 zflag if zflag is not None else 0.0)

            def gram_exe(paths):
                """(executed lane flops per chain-Gram, share of low-rank Grams) from the
                path counts the kernel reported (gst_gram_counts)."""
                tot = paths["low_rank"] + paths["mfma"]
                if tot <= 0:
                    return float("nan"), float("nan")
                f_lr = paths["low_rank"] / tot
                return f_lr * pf["low_rank"] + (1 - f_lr) * pf["mfma"], f_lr

            g_exe, g_lr = gram_exe(stage_ms["gram_gram_paths"])
            h_exe = g_exe + exe["tm_elim"] + exe["hyper_chol"]
            h_fix = g_alg + 12 * m ** 3 / 3
            stage_rep = {
                "source": "stage-masked launches of this run (HIP events), fixed cost "
                          f"{fx * 1e3:.1f} us/sweep subtracted; Gram paths counted by the "
                          "kernel (gst_gram_counts)",
                "gram": {"ms_per_sweep": t_gram,
                         "paths": stage_ms["gram_gram_paths"],
                         "low_rank_share": g_lr,
                         "executed_lane_flop_per_chain_gram": {
                             "low_rank_valu": pf["low_rank"], "mfma": pf["mfma"],
                             "flagged_toas_mean": zflag},
                         "tflops_executed": (g_exe + exe["tm_elim"]) * C / (t_gram * 1e-3) / 1e12,
                         "tflops_algorithmic": (g_alg + exe["tm_elim"]) * C / (t_gram * 1e-3) / 1e12,
                         "pipe": ("VALU (low-rank: class Grams + rank-1 updates)"
                                  if g_lr > 0.5 else "fp64 MFMA 16x16x4"),
                         "what": "Gram T^T N^-1 [T|r] + timing-model elimination; low-rank "
                                 "path on the VALU, n-TOA path on the fp64 MFMA (DESIGN.md 4)"},
                "gram_cholesky": {"ms_per_sweep": t_hyp,
                                  "tflops_executed": h_exe * C / (t_hyp * 1e-3) / 1e12,
                                  "tflops_fixed_formula": h_fix * C / (t_hyp * 1e-3) / 1e12,
                                  "what": "whole red-noise block: Gram + 11 likelihood "
                                          "factorisations (VALU: register-resident LDL^T)"},
            }
            for v in stage_rep.values():
                if isinstance(v, dict):
                    for k2 in [k for k in v if k.startswith("tflops")]:
                        v[k2.replace("tflops", "frac")] = v[k2] / FP64_PEAK_TFLOPS
        ess_ps, reason = None, None
        if ess is None:
            reason = "no ESS window (config 5: 155 ms per sweep)" if ess_win <= 0 else "n/a"
        else:
            # ESS over every chain of the job / the window's wall time (max over ranks)
            ess_ps, reason = ess_rate(ess, rhat, win_s)
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "chain-sweeps/s",
            "n_gpus": world,
            "steps": K,
            "warmup": W,
            "ms_per_step": elapsed / K * 1e3,
            "higher_is_better": True,
            "scaling": wl["scaling"],
            "vs_baseline": None,
            "dtype": "f64",
            "data": wl["data"],
            "config": {"workload": wl["desc"], "baseline_config": args.config,
                       "chains_per_gpu": C, "chains_total": C * world, "n_toa": n,
                       "basis_cols": m, "datasets_per_gpu": len(wl["ptas"]),
                       "record_every": 1,
                       "parallelism": f"independent chains sharded over {world} GPU(s); "
                                      "RCCL only for the final gather of chain draws to rank 0"},
            "ess_per_sec": ess_ps,
            "ess_per_sec_reason": reason,
            # config 4: the same per outlier model of the run_sims grid (each model's chains
            # share the window's wall time with the others')
            "ess_by_model": None if by_group is None else {
                g: dict(zip(("ess_per_sec", "reason"), ess_rate(e, r, win_s)),
                        rhat_max=r,
                        # the model's datasets whose every split R-hat <= RHAT_OK (bimodal
                        # posteriors put the others' chains in different modes):
                        # their summed ESS of the slowest parameter over the window's time
                        converged_datasets={
                            "datasets": conv_group[g][1], "of": conv_group[g][2],
                            "ess_per_sec": (min(v for v in conv_group[g][0].values() if v > 0)
                                            / win_s if conv_group[g][1] else None)})
                for g, (e, r) in sorted(by_group.items())},
            "ess_window": {"burn_in_sweeps": W + K + burn, "sweeps": ess_win, "thin": thin,
                           "seconds": win_s, "chains": C * world,
                           "ess_total": ess, "rhat_max": rhat},
            "shards": [[int(a), int(b)] for a, b in shards],   # global chain ids per rank
            "chains_with_status": int(s_vec[0]),
            "chains_floor_draw": ({"ess_window_chains": int(s_vec[3]),
                                   "ess_window_draws": int(s_vec[4]),
                                   "ess_window_draws_per_chain_sweep":
                                       float(s_vec[4]) / (C * world * ess_win),
                                   "since_start_chains": int(s_vec[1]),
                                   "since_start_draws": int(s_vec[2]),
                                   "what": "b draws at the SVD noise floor (include/gst.h): "
                                           "in the ESS window (stationary) and cumulative "
                                           "since the prior-draw start (warmup + timed)"}
                                  if ess_win > 0 else
                                  {"since_start_chains": int(s_vec[1]),
                                   "since_start_draws": int(s_vec[2])}),
            "kernel_ms": kernel_ms,
            # the persistent kernel is bound by VALU issue and the latency of the
            # factorisations' step-to-step LDS hand-offs (on config 2 its
            # Gram is the low-rank VALU update, so the PMC counts ~no MFMA work: roofline
            # ["gram_paths"] and ["mfma_pmc"]); its roofline is the fp64 peak, which MFMA and
            # VALU share on MI355X.  The large path's Gram is MFMA-bound.
            "roofline": {"bound": "mfma" if large else "valu-latency",
                         "peak_kind": "fp64 dense (MFMA = VALU rate on MI355X)",
                         "achieved": achieved, "peak": FP64_PEAK_TFLOPS,
                         "unit": "TFLOP/s", "frac": achieved / FP64_PEAK_TFLOPS,
                         "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": "lg_gram (per-launch HIP events)" if large else
                                   "gst_sweep_kernel (persistent, whole launch, HIP events)",
                         "algorithmic_flop_per_chain_sweep": algorithmic_flops(n_eff, m),
                         "executed_flop_per_chain_sweep": exe,
                         "per_toa_pass": toa,
                         "gram_paths": (None if gram_paths is None else
                                        dict(gram_paths, what="chain-Grams of the timed "
                                             "region by path (gst_gram_counts): persistent "
                                             "low-rank (VALU) / persistent MFMA / large-path "
                                             "MFMA")),
                         "mfma_pmc": pmc_mfma(pmc2) if not large else None,
                         "stages": stage_rep},
            "cpu_baseline": cpu,
        }
        if stages:
            out["stages"] = stages
        print(json.dumps(out), flush=True)
    ns.close()
    dist.finalize()
    return 0


if __name__ == "__main__":
    sys.exit(main())
