"""Pack the J1713+0747 dataset (TOAs, errors, fitted par values, red.txt) into an npz.

Runs ONLY in the build container (it reads `/root/reference`); the parsing itself is the
package's runtime tempo2 reader (gibbs_student_t_amd/partim.py), so any other pulsar's
par/tim pair loads the same way without this script.  The npz holds data, not source.

Reference files: J1713+0747.tim:3-132 (FORMAT 1 lines), J1713+0747.par:1-23, red.txt:1-130.
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from gibbs_student_t_amd import partim  # noqa: E402

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(__file__), "..", "gibbs_student_t_amd", "data",
                   "J1713+0747.npz")


def main():
    raw = partim.load_raw(os.path.join(REF, "J1713+0747.par"),
                          os.path.join(REF, "J1713+0747.tim"), os.path.join(REF, "red.txt"))
    np.savez(OUT, **partim.pack_npz(raw))
    print(f"wrote {OUT}: {len(raw['mjd_int'])} TOAs, {len(raw['fit'])} fitted params",
          file=sys.stderr)


if __name__ == "__main__":
    main()
