"""Extract the J1713+0747 dataset (TOAs, errors, fitted par values, red.txt) into an npz.

Runs ONLY in the build container (it reads `/root/reference`).  The npz holds data, not
source: per-TOA MJD (split into integer + fractional day to keep precision), error (us),
frequency (MHz); the par-file values of the fitted timing parameters; and the 130 numbers
of `red.txt`.  `gibbs_student_t_amd/data.py` reads the npz on any machine.

Reference files: J1713+0747.tim:3-132 (FORMAT 1 lines), J1713+0747.par:1-23, red.txt:1-130.
"""
import os
import sys
from decimal import Decimal

import numpy as np

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(__file__), "..", "gibbs_student_t_amd", "data",
                   "J1713+0747.npz")


def main():
    mjd_i, mjd_f, err, freq = [], [], [], []
    for line in open(os.path.join(REF, "J1713+0747.tim")):
        tok = line.split()
        if len(tok) < 5 or tok[0] in ("FORMAT", "MODE"):
            continue
        d = Decimal(tok[2])
        ip = int(d)
        mjd_i.append(ip)
        mjd_f.append(float(d - ip))
        freq.append(float(tok[1]))
        err.append(float(tok[3]))
    names, vals, fit = [], [], []
    for line in open(os.path.join(REF, "J1713+0747.par")):
        tok = line.split()
        if len(tok) < 2:
            continue
        key = tok[0]
        if key in ("RAJ", "DECJ"):
            parts = [float(x) for x in tok[1].split(":")]
            sign = -1.0 if tok[1].startswith("-") else 1.0
            deg = abs(parts[0]) + parts[1] / 60 + parts[2] / 3600
            v = sign * deg * (15.0 if key == "RAJ" else 1.0)
        else:
            try:
                v = float(tok[1])
            except ValueError:
                continue
        names.append(key)
        vals.append(v)
        fit.append(int(len(tok) > 2 and tok[2] == "1"))
    red = np.loadtxt(os.path.join(REF, "red.txt"))
    np.savez(OUT, mjd_int=np.array(mjd_i, dtype=np.int64), mjd_frac=np.array(mjd_f),
             toaerr_us=np.array(err), freq_mhz=np.array(freq),
             par_names=np.array(names), par_values=np.array(vals),
             par_fit=np.array(fit, dtype=np.int64), red=red)
    print(f"wrote {OUT}: {len(mjd_i)} TOAs, {sum(fit)} fitted params, red {red.shape}",
          file=sys.stderr)


if __name__ == "__main__":
    main()
