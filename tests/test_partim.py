"""The runtime tempo2 par/tim reader (gibbs_student_t_amd/partim.py).

* Against the reference's own J1713+0747 files (read in the build container only; the
  test skips where /root/reference is absent): the reader reproduces the packed
  data/J1713+0747.npz the sampler's J1713 dataset is built from, array for array.
* A synthetic pulsar written by the test (comments, commands, flags, INCLUDE, sexagesimal
  coordinates) round-trips.
Parity with tempo2 itself (clock corrections, barycentring, the design matrix) is
unpinned: tempo2 / libstempo are absent offline.
"""
import os

import numpy as np
import pytest

from gibbs_student_t_amd import data, partim

REF = "/root/reference"


@pytest.mark.skipif(not os.path.exists(os.path.join(REF, "J1713+0747.tim")),
                    reason="reference data files are only in the build container")
def test_reader_reproduces_packed_j1713():
    raw = partim.load_raw(os.path.join(REF, "J1713+0747.par"),
                          os.path.join(REF, "J1713+0747.tim"), os.path.join(REF, "red.txt"))
    packed = partim.pack_npz(raw)
    want = np.load(data.J1713_NPZ, allow_pickle=False)
    assert sorted(packed) == sorted(want.files)
    for k in want.files:
        np.testing.assert_array_equal(packed[k], want[k], err_msg=k)
    assert raw["name"] == "J1713+0747" and len(raw["fit"]) == 13


def test_synthetic_partim_round_trip(tmp_path):
    sub = tmp_path / "more.tim"
    sub.write_text("FORMAT 1\n t3 820.0 55001.000000000000000000001 1.5 ao -be GUPPI\n")
    (tmp_path / "p.tim").write_text(
        "FORMAT 1\nMODE 1\nC a comment line\n# another\n"
        " t1 1440.0 55000.123456789012345678 0.25 gbt -fe L-wide -be GUPPI\n"
        "JUMP\n"
        " t2 1440.0 55000.5 0.30 gbt\n"
        "INCLUDE more.tim\n")
    (tmp_path / "p.par").write_text(
        "PSRJ  J0000+0000\nRAJ   -01:30:00.0  1  1e-9\nDECJ  -10:30:00.0 1\n"
        "F0 100.5 1 1e-12\nF1 -1.0D-15 1\nPEPOCH 55000\nBINARY DD\n")
    tim = partim.read_tim(str(tmp_path / "p.tim"))
    assert tim.n == 3 and tim.site == ["gbt", "gbt", "ao"]
    np.testing.assert_array_equal(tim.mjd_int, [55000, 55000, 55001])
    assert abs(tim.mjd_frac[0] - 0.123456789012345678) < 1e-17
    assert tim.flags[0] == {"fe": "L-wide", "be": "GUPPI"} and tim.flags[1] == {}
    np.testing.assert_array_equal(tim.toaerr_us, [0.25, 0.30, 1.5])
    par = partim.read_par(str(tmp_path / "p.par"))
    assert par.name == "J0000+0000" and par.fitted == ["RAJ", "DECJ", "F0", "F1"]
    assert par.values["RAJ"] == pytest.approx(-22.5) and par.values["DECJ"] == pytest.approx(-10.5)
    assert par.values["F1"] == -1.0e-15 and par.values["BINARY"] == "DD"
    assert par.uncertainty["F0"] == 1e-12 and par.uncertainty["PEPOCH"] is None
    # the sampler's dataset builder accepts any reader output
    raw = partim.load_raw(str(tmp_path / "p.par"), str(tmp_path / "p.tim"))
    M = data.design_matrix(tim.mjd, raw["par"], raw["fit"])
    assert M.shape == (3, 1 + 4)


@pytest.mark.skipif(not os.path.exists(os.path.join(REF, "J1713+0747.tim")),
                    reason="reference data files are only in the build container")
def test_load_partim_equals_packed_dataset():
    """The runtime loader builds the same J1713 dataset as the packed npz (bit for bit)."""
    a = data.j1713(seed=5, red_source="red.txt")
    b = data.load_partim(os.path.join(REF, "J1713+0747.par"),
                         os.path.join(REF, "J1713+0747.tim"), os.path.join(REF, "red.txt"),
                         seed=5, red_source="red.txt")
    for k in ("toas", "residuals", "toaerrs", "Mmat"):
        np.testing.assert_array_equal(getattr(a, k), getattr(b, k), err_msg=k)
