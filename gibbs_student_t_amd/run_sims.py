"""Simulation-study driver: the run_sims.py grid batched into GPU launches.

Reference: /root/reference/run_sims.py.  For each outlier fraction theta (:35-36) it
simulates a pulsar (simulate_data.py:10-39), loads the outlier and the no_outlier twin
(:44-53), runs the five outlier models (:86-107) for niter = 10000 sweeps from a prior
draw (:110-113) and saves every chain array after a 100-sweep burn-in (:118-124) to
``{outdir}/{model}/{theta}/{idx}/{chain,bchain,zchain,poutchain,thetachain,alphachain,
dfchain}.npy`` with outdir in {output_outlier, output_no_outlier} (:78,114).

Here the whole grid -- realisations x {outlier, no_outlier} x models -- is ONE batch of
datasets (gst_model_set_batch) and each (dataset, model) entry gets ``chains`` independent
chains, so the study runs as a few persistent kernel launches instead of
3 x 2 x 5 sequential single-chain Python loops.  Records stream to host ``.npy`` files
chunk by chunk (numpy memmaps), so HBM holds only one chunk of records.  With
``chains == 1`` the files have exactly the reference's shapes; otherwise a leading chain
axis is added (as ``Gibbs(nchains=...)`` does).  Multi-GPU: entries are sharded by rank
(contiguous blocks), chain ids stay global, so the output does not depend on the sharding.
"""
from __future__ import annotations

import argparse
import json
import os
import time
from dataclasses import dataclass, field

import numpy as np

from . import data as gdata
from .model import PTA

# run_sims.py:89-107
MODELS = {
    "vvh17": dict(model="vvh17", vary_df=False, theta_prior="uniform", vary_alpha=False,
                  alpha=1e10, pspin=0.00457),
    "uniform": dict(model="mixture", vary_df=True, theta_prior="uniform"),
    "beta": dict(model="mixture", vary_df=True, theta_prior="beta"),
    "gaussian": dict(model="gaussian", vary_df=True, theta_prior="beta"),
    "t": dict(model="t", vary_df=True, theta_prior="beta"),
}
OUTDIRS = {"outlier": "output_outlier", "no_outlier": "output_no_outlier"}  # run_sims.py:78
CHAIN_FILES = (("x", "chain"), ("b", "bchain"), ("z", "zchain"), ("pout", "poutchain"),
               ("theta", "thetachain"), ("alpha", "alphachain"), ("nu", "dfchain"))


@dataclass
class Entry:
    """One Gibbs object of the reference study: a dataset under one outlier model."""

    kind: str            # 'outlier' | 'no_outlier'
    theta: float         # simulated outlier fraction
    idx: int             # realisation id (run_sims.py:39 uses random.getrandbits(32))
    model: str           # key of MODELS
    pta: PTA
    dof: float | None = None
    meta: dict = field(default_factory=dict)

    @property
    def cfg(self):
        return MODELS[self.model]

    def outdir(self, root):
        tag = self.theta if self.dof is None else f"{self.theta}_t{self.dof:g}"
        return os.path.join(root, OUTDIRS[self.kind], self.model, str(tag), str(self.idx))


def build_grid(thetas=(0.05, 0.1, 0.15), realisations=1, models=tuple(MODELS),
               seed=2017, sigma_out=1e-6, red_source="powerlaw", dofs=(None,),
               kinds=("outlier", "no_outlier"), generator="host", device=0):
    """The study's entries in a fixed global order (realisation-major).

    ``generator="host"``: realisation k at outlier fraction theta and white-noise dof uses
    data.simulate_data with a seed derived from (seed, k, theta, dof).  ``"device"``: every
    (k, theta, dof) dataset of the grid is drawn in ONE gst_simulate launch (simulate.py),
    dataset id = its position in that order.  Either way entry lists built on different
    ranks agree.
    """
    if generator == "device":
        return _grid_on_device(thetas, realisations, models, seed, sigma_out, red_source,
                               dofs, kinds, device)
    if generator != "host":
        raise ValueError("generator must be 'host' or 'device'")
    entries = []
    for k in range(realisations):
        for ti, theta in enumerate(thetas):
            for di, dof in enumerate(dofs):
                sd = int(np.random.SeedSequence([seed, k, ti, di]).generate_state(1)[0])
                out, clean = gdata.simulate_data(sd, theta=theta, sigma_out=sigma_out,
                                                 red_source=red_source, dof=dof)
                pair = {"outlier": out, "no_outlier": clean}
                for kind in kinds:
                    pta = PTA(pair[kind])
                    for mdl in models:
                        entries.append(Entry(kind, float(theta), sd, mdl, pta, dof,
                                             {"z_true": out.meta["z_true"]}))
    return entries


def _grid_on_device(thetas, realisations, models, seed, sigma_out, red_source, dofs, kinds,
                    device):
    from . import simulate
    raw = gdata.load_j1713_raw()
    mjd = raw["mjd_int"].astype(np.float64) + raw["mjd_frac"]
    toas = mjd * gdata.DAY_SEC
    M = gdata.design_matrix(mjd, raw["par"], raw["fit"])
    combos = [(k, float(theta), dof) for k in range(realisations) for theta in thetas
              for dof in dofs]
    red = raw["red"] * gdata.DAY_SEC if red_source == "red.txt" else None
    sim = simulate.simulate_batch(
        toas, M, len(combos), seed=seed, theta=[c[1] for c in combos], sigma_out=sigma_out,
        dof=[0.0 if c[2] is None else float(c[2]) for c in combos], red=red,
        clean="no_outlier" in kinds, device=device)
    prs = simulate.pairs(toas, M, sim, name="J1713+0747", freqs=raw["freq_mhz"])
    entries = []
    for i, ((k, theta, dof), (out, clean)) in enumerate(zip(combos, prs)):
        pair = {"outlier": out, "no_outlier": clean}
        for kind in kinds:
            pta = PTA(pair[kind])
            for mdl in models:
                entries.append(Entry(kind, theta, i, mdl, pta, dof,
                                     {"z_true": out.meta["z_true"], "generator": "device"}))
    return entries


# A record is "in the all-outlier state" when at least half of its TOAs are flagged
# (sum z >= n / 2).  vvh17 chains start there (z = 1 with alpha fixed at 1e10, gibbs.py:44-51:
# every TOA is effectively removed, b is drawn from its prior, q ~ 1 keeps z = 1).  The
# reference's chains leave within ~100 sweeps through its SVD draw's rounding floor at
# cond(Sigma) ~ 1e22 (gibbs.py:169-180), which the HIP path reproduces (include/gst.h
# gst_sweep; with the exact draw a chain stays for thousands of sweeps).
# The study still reports the fraction of such records per entry and warns when a vvh17
# entry keeps any.
TRAP_WARN_FRAC = 0.01


def initial_state(entry: Entry, chains: int, gid0: int, seed: int, nst: int,
                  vvh17_start: str = "reference"):
    """Prior draw per chain (run_sims.py:111) and the gibbs.py:29-51 latent initial state.

    ``vvh17_start="clean"`` (opt-in) starts vvh17 chains with no TOA flagged (z = 0) instead
    of the reference's all-outlier start (z = 1, gibbs.py:50-51)."""
    if vvh17_start not in ("reference", "clean"):
        raise ValueError("vvh17_start must be 'reference' or 'clean'")
    pta, cfg = entry.pta, entry.cfg
    n, m = pta.T.shape
    lo = np.array([p.pmin for p in pta.params])
    hi = np.array([p.pmax for p in pta.params])
    x = np.stack([np.random.default_rng([seed, gid0 + c]).uniform(lo, hi)
                  for c in range(chains)])
    z0 = 1.0 if cfg["model"] in ("t", "mixture", "vvh17") else 0.0
    if cfg["model"] == "vvh17" and vvh17_start == "clean":
        z0 = 0.0
    a0 = 1.0 if cfg.get("vary_alpha", True) else float(cfg.get("alpha", 1e10))
    z = np.zeros((chains, nst))
    z[:, :n] = z0
    alpha = np.ones((chains, nst))
    alpha[:, :n] = a0
    return dict(x=x, b=np.zeros((chains, m)), z=z, alpha=alpha, pout=np.zeros((chains, nst)),
                theta=np.full(chains, float(cfg.get("m", 0.01))),
                nu=np.full(chains, float(cfg.get("tdf", 4))))


class Study:
    """A batch of entries x ``chains`` chains on one GPU (one NativeSampler).

    ``vvh17_start``: "reference" (default) starts vvh17 chains as gibbs.py:50-51 does (z = 1);
    "clean" (opt-in) with no TOA flagged."""

    def __init__(self, entries, chains=1, device=0, seed=1, entry0=0,
                 vvh17_start="reference"):
        from .native import NativeSampler
        self.entries = list(entries)
        self.chains = int(chains)
        self.seed = int(seed)
        self.entry0 = int(entry0)          # global index of entries[0] (sharding)
        self.ns = NativeSampler([e.pta for e in self.entries],
                                [e.cfg for e in self.entries], device)
        E = len(self.entries)
        self.ns.alloc(E * self.chains, dataset=np.repeat(np.arange(E), self.chains))
        nst = self.ns.n
        parts = [initial_state(e, self.chains, (self.entry0 + i) * self.chains, self.seed, nst,
                               vvh17_start)
                 for i, e in enumerate(self.entries)]
        self.ns.set_state(**{k: np.concatenate([p[k] for p in parts]) for k in parts[0]})
        self.sweeps_done = 0
        self.vvh17_start = vvh17_start
        self.trapped = None

    @property
    def chain0(self):
        return self.entry0 * self.chains

    def run(self, niter, burn=100, outdir=None, chunk=500, record_every=1, keys=None,
            progress=None):
        """Sample ``niter`` sweeps; write [burn:] records per entry under ``outdir``.

        Returns ``(records or None, seconds)``: without ``outdir`` the post-burn records
        are returned as host arrays ``{key: [E, chains, nrec, ...]}``.
        """
        ns, E, C = self.ns, len(self.entries), self.chains
        keys = [k for k, _ in CHAIN_FILES] if keys is None else list(keys)
        every = max(1, int(record_every))
        nrec_total = (niter + every - 1) // every
        first = (burn + every - 1) // every            # first kept record index
        keep = max(0, nrec_total - first)
        shapes = {"x": (ns.P,), "b": (ns.m,), "z": (ns.n,), "alpha": (ns.n,),
                  "pout": (ns.n,), "theta": (), "nu": ()}
        sinks = self._open_sinks(outdir, keys, keep, shapes)
        chunk = max(every, (int(chunk) // every) * every)
        # all-outlier-state counts of the kept records, per chain (from z when recorded,
        # else from theta: for vvh17's uniform theta prior theta ~ Beta(sum z + 1, n - sum z
        # + 1), so theta >= 1/2 is the same state)
        tdev = ns.tdev
        import torch
        n_of = torch.tensor(np.repeat([e.pta.n for e in self.entries], C), device=tdev,
                            dtype=torch.float64)
        tmask = (torch.arange(ns.n, device=tdev)[None, :] < n_of[:, None]).to(torch.float64)
        trap_src = "z" if "z" in keys else ("theta" if "theta" in keys else None)
        trap_cnt = torch.zeros(E * C, dtype=torch.float64, device=tdev)
        trap_last = torch.zeros(E * C, dtype=torch.float64, device=tdev)
        t0 = time.perf_counter()
        done, ri = 0, 0
        while done < niter:
            k = min(chunk, niter - done)
            kr = (k + every - 1) // every
            rec = ns.alloc_records(kr, keys=keys)
            ns.sweep(k, records=rec, record_every=every, seed=self.seed,
                     sweep0=self.sweeps_done, chain0=self.chain0)
            self.sweeps_done += k
            lo = max(ri, first)
            if lo < ri + kr:
                for key in keys:
                    host = rec[key][:, lo - ri:].cpu().numpy()
                    host = host.reshape((E, C) + host.shape[1:])
                    self._write(sinks, key, host, lo - first)
                if trap_src == "z":
                    zs = (rec["z"][:, lo - ri:] * tmask[:, None, :]).sum(-1)
                    st = (zs >= 0.5 * n_of[:, None]).to(torch.float64)
                elif trap_src == "theta":
                    st = (rec["theta"][:, lo - ri:] >= 0.5).to(torch.float64)
                if trap_src:
                    trap_cnt += st.sum(1)
                    trap_last = st[:, -1]
            done += k
            ri += kr
            if progress:
                progress(done, niter, time.perf_counter() - t0)
        ns.synchronize()
        secs = time.perf_counter() - t0
        self.trapped = self._trap_summary(trap_src, trap_cnt.cpu().numpy(),
                                          trap_last.cpu().numpy(), keep)
        if outdir is not None and self.trapped:
            with open(os.path.join(outdir, f"trapped_entries_{self.entry0}.json"), "w") as f:
                json.dump(self.trapped, f, indent=1)
        return self._close_sinks(sinks, outdir), secs

    def _trap_summary(self, src, cnt, last, keep):
        """Per entry: fraction of kept records (and of chains at the last record) in the
        all-outlier state; a warning for vvh17 entries above TRAP_WARN_FRAC."""
        if src is None or keep <= 0:
            return None
        E, C = len(self.entries), self.chains
        out = []
        for i, e in enumerate(self.entries):
            frac = float(cnt[i * C:(i + 1) * C].sum() / (C * keep))
            end = float(last[i * C:(i + 1) * C].mean())
            row = {"entry": self.entry0 + i, "kind": e.kind, "theta": e.theta, "idx": e.idx,
                   "model": e.model, "source": src, "trapped_record_frac": frac,
                   "trapped_chain_frac_end": end}
            if e.model == "vvh17":
                row["vvh17_start"] = self.vvh17_start
            if e.model == "vvh17" and frac > TRAP_WARN_FRAC:
                row["warning"] = (
                    f"{frac:.1%} of the kept records sit in the all-outlier state (sum z >= "
                    f"n/2; start '{self.vvh17_start}'): burn in longer (DESIGN.md section 3)")
                import sys
                print(f"run_sims WARNING entry {self.entry0 + i} ({e.kind}, theta={e.theta}, "
                      f"vvh17): {row['warning']}", file=sys.stderr, flush=True)
            out.append(row)
        return out

    # ---- record sinks -------------------------------------------------------------------
    def _open_sinks(self, outdir, keys, keep, shapes):
        E, C = len(self.entries), self.chains
        sinks = {}
        for key in keys:
            if outdir is None:
                sinks[key] = np.zeros((E, C, keep) + shapes[key])
                continue
            fname = dict(CHAIN_FILES)[key]
            per = []
            for e in self.entries:
                d = e.outdir(outdir)
                os.makedirs(d, exist_ok=True)
                tail = (e.pta.n,) if key in ("z", "alpha", "pout") else shapes[key]
                shape = ((C,) if C > 1 else ()) + (keep,) + tail
                per.append(np.lib.format.open_memmap(os.path.join(d, fname + ".npy"),
                                                     mode="w+", dtype=np.float64,
                                                     shape=shape))
            sinks[key] = per
        return sinks

    def _write(self, sinks, key, host, at):
        s = sinks[key]
        w = host.shape[2]
        if isinstance(s, np.ndarray):
            s[:, :, at:at + w] = host
            return
        for i, (mm, e) in enumerate(zip(s, self.entries)):
            blk = host[i]
            if mm.ndim >= 2 and key in ("z", "alpha", "pout"):
                blk = blk[..., :e.pta.n]
            if self.chains == 1:
                mm[at:at + w] = blk[0]
            else:
                mm[:, at:at + w] = blk

    def _close_sinks(self, sinks, outdir):
        if outdir is None:
            return sinks
        for per in sinks.values():
            for mm in per:
                mm.flush()
        return None

    def close(self):
        self.ns.close()


def summarise(entries, recs, chains):
    """Per-entry posterior summaries (means, ESS, R-hat) from returned records."""
    from . import diag
    out = []
    names = [p.name.split("_", 1)[1] for p in entries[0].pta.params]
    for i, e in enumerate(entries):
        row = {"kind": e.kind, "theta": e.theta, "idx": e.idx, "model": e.model,
               "dof": e.dof, "n": e.pta.n}
        for j, nm in enumerate(names):
            s = recs["x"][i, :, :, j]
            row[f"mean_{nm}"] = float(s.mean())
            row[f"ess_{nm}"] = float(diag.bulk_ess(s)) if chains > 1 or s.shape[1] > 8 else None
            if chains > 1:
                row[f"rhat_{nm}"] = float(diag.split_rhat(s))
        if "theta" in recs:
            row["mean_theta"] = float(recs["theta"][i].mean())
        if "z" in recs and e.kind == "outlier":
            zt = e.meta["z_true"]
            zhat = recs["pout"][i, :, :, :e.pta.n].mean(axis=(0, 1)) if "pout" in recs else None
            if zhat is not None and e.cfg["model"] in ("mixture", "vvh17"):
                row["outlier_auc_like"] = float(np.mean(zhat[zt == 1]) - np.mean(zhat[zt == 0])) \
                    if zt.any() and (~zt.astype(bool)).any() else None
        out.append(row)
    return out


def main(argv=None):
    ap = argparse.ArgumentParser(description="run_sims.py study grid on the GPU")
    ap.add_argument("--thetas", type=float, nargs="+", default=[0.05, 0.1, 0.15])
    ap.add_argument("--realisations", type=int, default=1)
    ap.add_argument("--models", nargs="+", default=list(MODELS))
    ap.add_argument("--dofs", type=float, nargs="*", default=[])
    ap.add_argument("--chains", type=int, default=1)
    ap.add_argument("--niter", type=int, default=10000)       # run_sims.py:112
    ap.add_argument("--burn", type=int, default=100)          # run_sims.py:118
    ap.add_argument("--chunk", type=int, default=500)
    ap.add_argument("--record-every", type=int, default=1)
    ap.add_argument("--outdir", default=None)
    ap.add_argument("--seed", type=int, default=2017)
    ap.add_argument("--generator", choices=("device", "host"), default="device",
                    help="draw the grid's datasets in one GPU launch (default) or per "
                         "dataset with NumPy")
    ap.add_argument("--red-source", choices=("powerlaw", "red.txt"), default="powerlaw")
    ap.add_argument("--vvh17-start", choices=("reference", "clean"), default="reference",
                    help="vvh17 initial outlier flags: the reference's z = 1 (gibbs.py:50-51, "
                         "default) or z = 0")
    args = ap.parse_args(argv)
    from . import dist
    rank, local, world = dist.init()
    dofs = tuple([None] + list(args.dofs)) if args.dofs else (None,)
    entries = build_grid(args.thetas, args.realisations, tuple(args.models), args.seed,
                         red_source=args.red_source, dofs=dofs, generator=args.generator,
                         device=local)
    per = (len(entries) + world - 1) // world
    mine = entries[rank * per:(rank + 1) * per]
    if not mine:
        dist.finalize()
        return
    st = Study(mine, chains=args.chains, device=local, seed=args.seed, entry0=rank * per,
               vvh17_start=args.vvh17_start)
    recs, secs = st.run(args.niter, burn=args.burn, outdir=args.outdir, chunk=args.chunk,
                        record_every=args.record_every)
    total = len(mine) * args.chains * args.niter
    print(json.dumps({"rank": rank, "entries": len(mine), "chains": args.chains,
                      "sweeps": args.niter, "vvh17_start": args.vvh17_start, "seconds": secs,
                      "chain_sweeps_per_s": total / secs}), flush=True)
    for row in st.trapped or []:
        if row["trapped_record_frac"] > 0:
            print(json.dumps({"rank": rank, "trapped": row}), flush=True)
    if recs is not None and rank == 0:
        for row in summarise(mine, recs, args.chains):
            print(json.dumps(row))
    st.close()
    dist.finalize()


if __name__ == "__main__":
    main()
