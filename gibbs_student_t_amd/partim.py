"""tempo2 ``.par`` / ``.tim`` readers: the pulsar inputs of the reference's study.

The reference loads pulsars with ``enterprise.pulsar.Pulsar(par, tim)`` (run_sims.py:47,51;
gibbs_likelihood.ipynb cell 3), i.e. tempo2 through libstempo.  Neither exists offline, so
this module reads the two text formats itself and hands the sampler what it needs from
them -- TOA epochs, error bars, observing frequencies, the fitted timing-model parameters --
leaving the timing model's design matrix to ``data.design_matrix`` (an analytic
approximation; parity with tempo2 is *unpinned*, see data.py).

Formats (as the reference's own files use them, J1713+0747.tim:1-132, J1713+0747.par:1-23):

* tim, ``FORMAT 1``: one TOA per line, ``name freq_MHz MJD err_us site [-flag value ...]``;
  command lines (``FORMAT``, ``MODE``, ``EFAC``, ``JUMP`` ...) and comments (``C ...``,
  ``# ...``) carry no TOA; ``INCLUDE file`` pulls in another tim file relative to this one.
  MJDs keep their full precision as an integer day plus a fractional day (a float64 MJD
  alone would lose ~1 us).
* par: ``NAME value [fit-flag [uncertainty]]``; RAJ / DECJ are sexagesimal (hours /
  degrees) and are returned in degrees; non-numeric values (``BINARY DD``) are kept as
  strings; the fit flag ``1`` marks the parameters tempo2 fits (the timing-model columns).
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from decimal import Decimal, InvalidOperation

import numpy as np

TIM_COMMANDS = {"FORMAT", "MODE", "EFAC", "EQUAD", "EMAX", "EMIN", "FMAX", "FMIN", "JUMP",
                "TIME", "PHASE", "SKIP", "NOSKIP", "END", "TRACK", "INFO", "SIGMA", "INCLUDE"}


@dataclass
class Tim:
    """TOAs of a tempo2 FORMAT 1 file (file order)."""

    names: list
    freq_mhz: np.ndarray
    mjd_int: np.ndarray        # integer day
    mjd_frac: np.ndarray       # fractional day, exact to ~1e-16 day
    toaerr_us: np.ndarray
    site: list
    flags: list = field(default_factory=list)   # per TOA: {flag: value}

    @property
    def n(self):
        return len(self.mjd_int)

    @property
    def mjd(self):
        return self.mjd_int.astype(np.float64) + self.mjd_frac


def _split_mjd(tok: str):
    try:
        d = Decimal(tok)
    except InvalidOperation as e:
        raise ValueError(f"bad MJD {tok!r}") from e
    i = int(d)
    return i, float(d - i)


def read_tim(path: str) -> Tim:
    """Parse a tempo2 FORMAT 1 tim file (following INCLUDE lines)."""
    out = dict(names=[], freq=[], mi=[], mf=[], err=[], site=[], flags=[])

    def parse(fn, depth):
        if depth > 8:
            raise ValueError("INCLUDE nesting too deep")
        with open(fn) as fh:
            for ln, line in enumerate(fh, 1):
                s = line.strip()
                if not s or s.startswith(("#", "C ")) or s == "C":
                    continue
                tok = s.split()
                key = tok[0].upper()
                if key == "INCLUDE":
                    parse(os.path.join(os.path.dirname(fn), tok[1]), depth + 1)
                    continue
                if key in TIM_COMMANDS:
                    continue
                if len(tok) < 5:
                    raise ValueError(f"{fn}:{ln}: TOA line needs name freq mjd err site")
                mi, mf = _split_mjd(tok[2])
                fl = {}
                rest = tok[5:]
                for k in range(0, len(rest) - 1, 2):
                    if rest[k].startswith("-"):
                        fl[rest[k][1:]] = rest[k + 1]
                out["names"].append(tok[0])
                out["freq"].append(float(tok[1]))
                out["mi"].append(mi)
                out["mf"].append(mf)
                out["err"].append(float(tok[3]))
                out["site"].append(tok[4])
                out["flags"].append(fl)

    parse(path, 0)
    return Tim(names=out["names"], freq_mhz=np.array(out["freq"]),
               mjd_int=np.array(out["mi"], dtype=np.int64), mjd_frac=np.array(out["mf"]),
               toaerr_us=np.array(out["err"]), site=out["site"], flags=out["flags"])


def _sexagesimal(v: str, hours: bool) -> float:
    parts = [float(x) for x in v.split(":")]
    sign = -1.0 if v.strip().startswith("-") else 1.0
    deg = abs(parts[0]) + (parts[1] if len(parts) > 1 else 0.0) / 60 \
        + (parts[2] if len(parts) > 2 else 0.0) / 3600
    return sign * deg * (15.0 if hours else 1.0)


@dataclass
class Par:
    """Parameters of a tempo2 par file, in file order."""

    values: dict               # name -> float (numeric) or str
    fit: dict                  # name -> bool (fit flag 1)
    uncertainty: dict          # name -> float or None

    @property
    def name(self):
        return str(self.values.get("PSRJ", self.values.get("PSR", "")))

    @property
    def fitted(self):
        return [k for k, f in self.fit.items() if f]

    def numeric(self):
        return {k: v for k, v in self.values.items() if isinstance(v, float)}


def read_par(path: str) -> Par:
    values, fit, unc = {}, {}, {}
    with open(path) as fh:
        for line in fh:
            tok = line.split()
            if not tok or tok[0].startswith("#") or tok[0] == "C":
                continue
            key = tok[0]
            if len(tok) < 2:
                continue
            raw = tok[1]
            if key in ("RAJ", "DECJ"):
                v = _sexagesimal(raw, hours=(key == "RAJ"))
            else:
                try:
                    v = float(raw.replace("D", "E")) if key != "PSRJ" else raw
                except ValueError:
                    v = raw
            values[key] = v
            fit[key] = len(tok) > 2 and tok[2] == "1" and isinstance(v, float)
            try:
                unc[key] = float(tok[3]) if len(tok) > 3 else None
            except ValueError:
                unc[key] = None
    return Par(values=values, fit=fit, uncertainty=unc)


def load_raw(par_path: str, tim_path: str, red_path: str | None = None) -> dict:
    """The raw dataset of one pulsar in the layout ``data.load_j1713_raw`` returns."""
    tim = read_tim(tim_path)
    par = read_par(par_path)
    numeric = par.numeric()
    raw = {"mjd_int": tim.mjd_int, "mjd_frac": tim.mjd_frac, "toaerr_us": tim.toaerr_us,
           "freq_mhz": tim.freq_mhz, "par": numeric,
           "fit": [k for k in par.fitted if k in numeric], "name": par.name}
    raw["red"] = np.loadtxt(red_path) if red_path else None
    return raw


def pack_npz(raw: dict) -> dict:
    """The arrays of ``data/J1713+0747.npz`` (tools/make_j1713_npz.py) from ``load_raw``."""
    names = list(raw["par"])
    return dict(mjd_int=raw["mjd_int"], mjd_frac=raw["mjd_frac"], toaerr_us=raw["toaerr_us"],
                freq_mhz=raw["freq_mhz"], par_names=np.array(names),
                par_values=np.array([raw["par"][k] for k in names]),
                par_fit=np.array([int(k in raw["fit"]) for k in names], dtype=np.int64),
                red=raw["red"] if raw["red"] is not None else np.zeros(0))


__all__ = ["Tim", "Par", "read_tim", "read_par", "load_raw", "pack_npz"]
