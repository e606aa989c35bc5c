"""The on-device RNG is standard Philox4x32-10: known-answer vectors (Salmon et al. SC'11,
Random123 kat_vectors) through the same header the kernel includes."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KAT = [
    ("00000000 00000000 00000000 00000000", "00000000 00000000",
     "6627e8d5 e169c58d bc57ac4c 9b00dbd8"),
    ("ffffffff ffffffff ffffffff ffffffff", "ffffffff ffffffff",
     "408f276d 41c83b0e a20bc7c6 6d5451fd"),
    ("243f6a88 85a308d3 13198a2e 03707344", "a4093822 299f31d0",
     "d16cfe09 94fdcceb 5001e420 24126ea1"),
]


@pytest.fixture(scope="module")
def kat_bin(tmp_path_factory):
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    out = tmp_path_factory.mktemp("kat") / "philox_kat"
    subprocess.run(["g++", "-O2", "-std=c++17", "-I",
                    os.path.join(ROOT, "gibbs_student_t_amd", "csrc"),
                    os.path.join(ROOT, "tools", "philox_kat.cpp"), "-o", str(out)], check=True)
    return str(out)


@pytest.mark.parametrize("ctr,key,want", KAT)
def test_philox_known_answers(kat_bin, ctr, key, want):
    out = subprocess.run([kat_bin] + ctr.split() + key.split(), capture_output=True,
                         text=True, check=True).stdout.strip()
    assert out == want
