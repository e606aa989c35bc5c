"""Device-side chain state and launches over the C ABI (libgst.so).

PyTorch-ROCm owns every chain buffer (``torch.empty(..., device='cuda')``); the library
receives raw ``data_ptr()`` values and the current HIP stream.  Nothing here computes a
sweep on the CPU: a missing library or device raises.
"""
from __future__ import annotations

import ctypes as ct

import numpy as np

from . import _abi
from .model import df_tables, hyper_white_indices

MODEL_CODES = {"gaussian": _abi.GST_MODEL_GAUSSIAN, "t": _abi.GST_MODEL_T,
               "mixture": _abi.GST_MODEL_MIXTURE, "vvh17": _abi.GST_MODEL_VVH17}
STATE_KEYS = ("x", "b", "z", "alpha", "pout", "theta", "nu")


def _torch():
    import torch
    return torch


def model_desc(pta, cfg: dict):
    """Build the gst_model_desc for a ``model.PTA`` and Gibbs kwargs (gibbs.py:9-11).

    Returns ``(desc, keepalive)``; keep ``keepalive`` referenced while ``desc`` is used.
    """
    names = [p.name for p in pta.params]
    P = len(names)
    hind, wind = hyper_white_indices(names)

    def role(suffix):
        for i, nm in enumerate(names):
            if nm.endswith("_" + suffix):
                return i
        return -1

    r = np.ascontiguousarray(pta.get_residuals()[0], dtype=np.float64)
    T = np.ascontiguousarray(pta.get_basis()[0], dtype=np.float64)
    n, m = T.shape
    A, B = df_tables(n)
    keep = {
        "T": T, "r": r,
        "err": np.ascontiguousarray(pta._toaerrs, dtype=np.float64),
        "ff": np.ascontiguousarray(pta.Ffreqs, dtype=np.float64),
        "pmin": np.array([p.pmin for p in pta.params], dtype=np.float64),
        "pmax": np.array([p.pmax for p in pta.params], dtype=np.float64),
        "hind": np.ascontiguousarray(hind, dtype=np.int32),
        "wind": np.ascontiguousarray(wind, dtype=np.int32),
        "A": np.ascontiguousarray(A, dtype=np.float64),
        "B": np.ascontiguousarray(B, dtype=np.float64),
    }
    # general white noise (ABI 3): per-backend parameters and ECORR basis columns
    nb = int(getattr(pta, "nbackend", 1))
    n_ec = int(getattr(pta, "n_ecorr", 0))
    if nb > 1 or n_ec:
        keep.update(
            bk=np.ascontiguousarray(pta.bidx, dtype=np.int32),
            efi=np.ascontiguousarray(pta.backend_param_indices("efac"), dtype=np.int32),
            eqi=np.ascontiguousarray(pta.backend_param_indices("log10_equad"), dtype=np.int32),
            eci=np.ascontiguousarray(pta.backend_param_indices("log10_ecorr"), dtype=np.int32),
            ecb=np.ascontiguousarray(pta.ecorr_backend, dtype=np.int32))
    dp = lambda a: a.ctypes.data_as(_abi._D)  # noqa: E731
    ip = lambda a: a.ctypes.data_as(_abi._I)  # noqa: E731
    model = cfg.get("model", "gaussian")
    if model not in MODEL_CODES:
        raise ValueError(f"unknown model {model!r}")
    if model == "vvh17" and cfg.get("pspin") is None:
        raise ValueError("model='vvh17' needs pspin")
    desc = _abi.ModelDesc(
        n=n, m=m, nfourier=pta.nfourier, ntm=pta.ntm, nparams=P,
        T=dp(keep["T"]), residuals=dp(keep["r"]), toaerrs=dp(keep["err"]),
        ffreqs=dp(keep["ff"]), tm_weight=float(pta.tm_weight),
        idx_efac=role("efac"), idx_equad=role("log10_equad"), idx_log10_A=role("log10_A"),
        idx_gamma=role("gamma"),
        efac_const=float(pta.efac_const if pta.efac_const is not None else 1.0),
        pmin=dp(keep["pmin"]), pmax=dp(keep["pmax"]),
        hyper_idx=ip(keep["hind"]), n_hyper=len(hind),
        white_idx=ip(keep["wind"]), n_white=len(wind),
        model=MODEL_CODES[model], vary_df=int(bool(cfg.get("vary_df", True))),
        vary_alpha=int(bool(cfg.get("vary_alpha", True))),
        theta_prior_beta=int(cfg.get("theta_prior", "beta") == "beta"),
        mprior=float(cfg.get("m", 0.01)),
        pspin=float(cfg.get("pspin") or 0.0),
        df_A=dp(keep["A"]), df_B=dp(keep["B"]),
    )
    if nb > 1 or n_ec:
        desc.nbackend = nb
        desc.backend = ip(keep["bk"])
        desc.efac_idx = ip(keep["efi"])
        desc.equad_idx = ip(keep["eqi"])
        desc.ecorr_idx = ip(keep["eci"])
        desc.n_ecorr = n_ec
        desc.ecorr_backend = ip(keep["ecb"]) if n_ec else None
    return desc, keep


class NativeSampler:
    """One HIP context + model + a batch of C chains resident on one GPU.

    ``pta``/``cfg`` may be lists: a batch of datasets (e.g. the run_sims.py grid of
    simulated pulsars x outlier models) sharing the basis shape and parameter set; each
    chain then names its dataset through ``alloc(C, dataset=...)``.  Per-TOA state and
    record arrays are laid out with row stride ``self.n`` = the largest n of the batch.
    """

    def __init__(self, pta, cfg: dict, device: int = 0, path: str = "auto"):
        torch = _torch()
        self.lib = _abi.load()
        if not torch.cuda.is_available():
            raise _abi.GstNativeError("no HIP device visible: the sampler runs only on GPU")
        self.device = int(device)
        self.tdev = torch.device("cuda", self.device)
        ptas = list(pta) if isinstance(pta, (list, tuple)) else [pta]
        cfgs = list(cfg) if isinstance(cfg, (list, tuple)) else [cfg] * len(ptas)
        if len(cfgs) != len(ptas):
            raise ValueError("one cfg per dataset (or a single shared cfg)")
        ctx = ct.c_void_p()
        _abi.check(self.lib, self.lib.gst_ctx_create(self.device, ct.byref(ctx)),
                   "gst_ctx_create")
        self.ctx = ctx
        if path not in _abi.PATHS:
            raise ValueError(f"path must be one of {sorted(_abi.PATHS)}")
        _abi.check(self.lib, self.lib.gst_set_path(self.ctx, _abi.PATHS[path]), "gst_set_path")
        self.ptas, self.cfgs = ptas, [dict(c) for c in cfgs]
        self.pta, self.cfg = ptas[0], self.cfgs[0]
        descs, self._keep = [], []
        for p_, c_ in zip(ptas, cfgs):
            d, k = model_desc(p_, c_)
            descs.append(d)
            self._keep.append(k)
        arr = (_abi.ModelDesc * len(descs))(*descs)
        _abi.check(self.lib, self.lib.gst_model_set_batch(self.ctx, arr, len(descs)),
                   "gst_model_set_batch")
        nd, nmax, stride = ct.c_int(), ct.c_int(), ct.c_int()
        _abi.check(self.lib, self.lib.gst_model_info(self.ctx, ct.byref(nd), ct.byref(nmax),
                                                     ct.byref(stride)), "gst_model_info")
        self.ndatasets = nd.value
        pth = ct.c_int()
        _abi.check(self.lib, self.lib.gst_get_path(self.ctx, ct.byref(pth)), "gst_get_path")
        self.path = {v: k for k, v in _abi.PATHS.items()}[pth.value]
        self.n_of = [int(p_.T.shape[0]) for p_ in ptas]
        self.n, self.m = nmax.value, int(ptas[0].T.shape[1])
        self.P = len(ptas[0].params)
        self.stride = stride.value
        self.C = 0
        self.state = None
        self.dataset = None

    def set_waves(self, waves="auto"):
        """Waves per chain of the persistent path's sampling launches (gst_set_waves):
        "auto" (two when C <= 2 x CUs), 1 or 2.  The draws are bitwise the same."""
        code = {"auto": 0, 1: 1, 2: 2}[waves]
        _abi.check(self.lib, self.lib.gst_set_waves(self.ctx, code), "gst_set_waves")

    def set_debug(self, poison: bool = False, large_gram: bool = False,
                  large_hyper: bool = False, exact_bdraw: bool = False,
                  mfma_gram: bool = False, epochs_lds: bool = False):
        """gst_set_debug: GST_DEBUG_POISON overwrites every chain's LDS and parked scratch
        with NaN at each sweep start (a check that no sweep reads stale state);
        GST_DEBUG_LARGE_GRAM / _HYPER force the large path's generic Gram / hyper kernels
        (tests compare them with the mid-size kernels); GST_DEBUG_EXACT_BDRAW draws b from
        Sigma exactly also beyond fp64 resolution (no SVD noise floor, include/gst.h);
        GST_DEBUG_MFMA_GRAM keeps the persistent kernel's Gram on the MFMA path (no low-rank
        Gram); GST_DEBUG_EPOCHS_LDS runs ECORR-epochs-first chains on the 256-thread lg_hyper<2>
        instead of the one-wave lg_hyper_ecr."""
        flags = ((_abi.DEBUG_POISON if poison else 0) | (_abi.DEBUG_LARGE_GRAM if large_gram else 0)
                 | (_abi.DEBUG_LARGE_HYPER if large_hyper else 0)
                 | (_abi.DEBUG_EXACT_BDRAW if exact_bdraw else 0)
                 | (_abi.DEBUG_MFMA_GRAM if mfma_gram else 0)
                 | (_abi.DEBUG_EPOCHS_LDS if epochs_lds else 0))
        _abi.check(self.lib, self.lib.gst_set_debug(self.ctx, flags), "gst_set_debug")

    # ---- state ---------------------------------------------------------------------
    def alloc(self, C: int, dataset=None):
        """Allocate C chains; ``dataset[c]`` is chain c's dataset index (default all 0)."""
        torch = _torch()
        f64 = dict(dtype=torch.float64, device=self.tdev)
        self.C = int(C)
        ds = np.zeros(C, dtype=np.int32) if dataset is None else \
            np.asarray(dataset, dtype=np.int32).reshape(C)
        if ds.size and (ds.min() < 0 or ds.max() >= self.ndatasets):
            raise ValueError(f"dataset indices must lie in [0, {self.ndatasets})")
        if dataset is None and self.ndatasets > 1:
            raise ValueError("several datasets: pass dataset= to alloc")
        if self.path == "large" and self.ndatasets > 1:
            # the large path stages one dataset's T per 16-chain group (Gram, T b)
            groups = [ds[i:i + 16] for i in range(0, C, 16)]
            if any(np.any(grp != grp[0]) for grp in groups):
                raise ValueError("large path with several datasets: every aligned group of "
                                 "16 chains must share one dataset")
        self.dataset_host = ds
        self.dataset = torch.as_tensor(ds).to(self.tdev)
        self.state = {
            "x": torch.zeros((C, self.P), **f64), "b": torch.zeros((C, self.m), **f64),
            "z": torch.zeros((C, self.n), **f64), "alpha": torch.ones((C, self.n), **f64),
            "pout": torch.zeros((C, self.n), **f64), "theta": torch.zeros(C, **f64),
            "nu": torch.zeros(C, **f64),
            "status": torch.zeros(C, dtype=torch.int32, device=self.tdev),
        }
        return self.state

    def set_state(self, **arrays):
        torch = _torch()
        for k, v in arrays.items():
            if v is None:
                continue
            t = self.state[k]
            src = torch.from_numpy(np.array(v, dtype=np.float64)).reshape(t.shape)
            t.copy_(src.to(self.tdev))

    def get_state(self):
        return {k: v.detach().cpu().numpy().copy() for k, v in self.state.items()}

    def _state_struct(self):
        s = self.state
        return _abi.State(*(ct.c_void_p(s[k].data_ptr()) for k in STATE_KEYS),
                          ct.c_void_p(s["status"].data_ptr()),
                          ct.c_void_p(self.dataset.data_ptr()))

    def alloc_records(self, nrec: int, keys=STATE_KEYS):
        torch = _torch()
        f64 = dict(dtype=torch.float64, device=self.tdev)
        shapes = {"x": (self.P,), "b": (self.m,), "z": (self.n,), "alpha": (self.n,),
                  "pout": (self.n,), "theta": (), "nu": ()}
        return {k: torch.empty((self.C, nrec) + shapes[k], **f64) for k in keys}

    # ---- launches ------------------------------------------------------------------
    def stream_ptr(self):
        torch = _torch()
        return ct.c_void_p(torch.cuda.current_stream(self.tdev).cuda_stream)

    def sweep(self, nsweeps: int, *, records=None, record_every: int = 1,
              mask: int = _abi.STAGE_ALL, seed: int = 0, sweep0: int = 0, chain0: int = 0,
              tape=None):
        """Launch ``nsweeps`` sweeps of all C chains.  ``records`` is a dict from
        ``alloc_records`` (or None); ``tape`` a device float64 tensor [C, nsweeps, stride]."""
        st = self._state_struct()
        rec = None
        if records is not None:
            nrec = next(iter(records.values())).shape[1]
            ptr = lambda k: ct.c_void_p(records[k].data_ptr()) if k in records else None  # noqa
            rec = _abi.Records(*(ptr(k) for k in STATE_KEYS), nrec)
        tp = None
        if tape is not None:
            if tuple(tape.shape) != (self.C, nsweeps, self.stride):
                raise ValueError(f"tape shape {tuple(tape.shape)} != "
                                 f"{(self.C, nsweeps, self.stride)}")
            tp = _abi.Tape(ct.c_void_p(tape.data_ptr()), self.stride)
        rc = self.lib.gst_sweep(self.ctx, ct.byref(st), ct.byref(rec) if rec else None,
                                ct.byref(tp) if tp else None, self.C, int(nsweeps),
                                int(sweep0), int(record_every if rec else 0), int(mask),
                                int(seed) & 0xFFFFFFFFFFFFFFFF, int(chain0), self.stream_ptr())
        _abi.check(self.lib, rc, "gst_sweep")

    def eval_lnlike(self):
        torch = _torch()
        ow = torch.empty(self.C, dtype=torch.float64, device=self.tdev)
        oh = torch.empty(self.C, dtype=torch.float64, device=self.tdev)
        st = self._state_struct()
        rc = self.lib.gst_eval_lnlike(self.ctx, ct.byref(st), self.C,
                                      ct.c_void_p(ow.data_ptr()), ct.c_void_p(oh.data_ptr()),
                                      self.stream_ptr())
        _abi.check(self.lib, rc, "gst_eval_lnlike")
        return ow.cpu().numpy(), oh.cpu().numpy()

    def synchronize(self):
        _abi.check(self.lib, self.lib.gst_sync(self.ctx, self.stream_ptr()), "gst_sync")

    def last_kernel_ms(self):
        ms = ct.c_double()
        _abi.check(self.lib, self.lib.gst_last_sweep_ms(self.ctx, ct.byref(ms)),
                   "gst_last_sweep_ms")
        return ms.value

    def set_timing(self, on: bool = True):
        """Per-kernel HIP-event timing of the large path (kernel_times())."""
        _abi.check(self.lib, self.lib.gst_set_timing(self.ctx, int(bool(on))), "gst_set_timing")

    def kernel_times(self):
        """{kind: (total ms, launches)} for the last launch with timing enabled."""
        k = len(_abi.KERNEL_KINDS)
        ms = (ct.c_double * k)()
        nl = (ct.c_int * k)()
        _abi.check(self.lib, self.lib.gst_kernel_times(self.ctx, ms, nl, k), "gst_kernel_times")
        return {name: (ms[i], nl[i]) for i, name in enumerate(_abi.KERNEL_KINDS)}

    def gram_counts(self, reset: bool = True):
        """Grams computed since the last reset, by path (include/gst.h gst_gram_counts):
        {"low_rank": persistent low-rank (VALU), "mfma": persistent fp64 MFMA,
        "large_mfma": large path fp64 MFMA} in chain-Grams; synchronises the device."""
        v = (ct.c_longlong * 3)()
        _abi.check(self.lib, self.lib.gst_gram_counts(self.ctx, v, int(bool(reset))),
                   "gst_gram_counts")
        return {"low_rank": int(v[0]), "mfma": int(v[1]), "large_mfma": int(v[2])}

    def close(self):
        if getattr(self, "ctx", None):
            self.lib.gst_ctx_destroy(self.ctx)
            self.ctx = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


def pack_tape(ref_tape: dict, sweeps, n: int, m: int, stride: int, nst: int | None = None):
    """Golden-fixture tape (tools/gen_golden.py fields) -> [len(sweeps), stride] rows.

    ``nst`` is the per-TOA row stride of the launch (the batch's largest n; default n)."""
    nst = n if nst is None else int(nst)
    rows = np.zeros((len(sweeps), stride))
    for k, i in enumerate(sweeps):
        row = rows[k]
        for stage, off, ns in (("white", _abi.TAPE_WHITE, 20), ("hyper", _abi.TAPE_HYPER, 10)):
            e = np.stack([ref_tape[f"{stage}_u"][i], ref_tape[f"{stage}_idx"][i].astype(float),
                          ref_tape[f"{stage}_xi"][i], ref_tape[f"{stage}_acc"][i]], axis=1)
            row[off:off + 4 * ns] = e.reshape(-1)
        o = _abi.TAPE_DELTA
        row[o:o + m] = np.nan_to_num(ref_tape["b_delta"][i])
        row[o + m] = ref_tape["beta"][i]
        row[o + m + 1:o + m + 1 + n] = ref_tape["z_u"][i]
        row[o + m + 1 + nst:o + m + 1 + nst + n] = ref_tape["gamma"][i]
        row[o + m + 1 + 2 * nst] = ref_tape["df_u"][i]
    return rows


def debug_variates(kind: str, a: float, n: int, b: float = 1.0, seed: int = 1, call: int = 0,
                   device: int = 0):
    """The kernel's own samplers (include/gst.h gst_debug_variates) -> float64 device tensor:
    kind "gamma" (gamma_mt), "beta" (the theta stage's two-gamma Beta), "gamma_slots" (the
    alpha stage's gamma_mt_slots<4>; n a multiple of 256)."""
    torch = _torch()
    lib = _abi.load()
    k = {"gamma": 0, "beta": 1, "gamma_slots": 2}[kind]
    out = torch.empty(int(n), dtype=torch.float64, device=f"cuda:{device}")
    with torch.cuda.device(device):
        st = torch.cuda.current_stream().cuda_stream
        rc = lib.gst_debug_variates(k, float(a), float(b), int(n), int(seed), int(call),
                                    ct.c_void_p(out.data_ptr()), ct.c_void_p(st))
    _abi.check(lib, rc, "gst_debug_variates")
    return out
