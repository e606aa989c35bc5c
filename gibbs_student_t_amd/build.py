"""Build libgst.so in-tree with hipcc for gfx950 (no JIT cache: the .so travels with the repo)."""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libgst.so")
SOURCES = [os.path.join(CSRC, f) for f in ("gst.hip", "gst_kernel.hpp", "gst_large.hpp",
                                            "philox.hpp")]
HEADER = os.path.join(ROOT, "include", "gst.h")


def hipcc():
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if cand and (os.path.isabs(cand) and os.path.exists(cand) or not os.path.isabs(cand)):
            return cand
    return "hipcc"


def up_to_date():
    if not os.path.exists(LIB):
        return False
    t = os.path.getmtime(LIB)
    return all(os.path.getmtime(s) <= t for s in SOURCES + [HEADER])


STAMPS_LIB = os.path.join(HERE, "libgst_stamps.so")


def build(force: bool = False, verbose: bool = True, stamps: bool = False) -> str:
    """Compile libgst.so (or the diagnostic libgst_stamps.so with per-stage cycle stamps)."""
    out = STAMPS_LIB if stamps else LIB
    if not force and not stamps and up_to_date():
        return LIB
    # -amdgpu-mfma-vgpr-form: keep the fp64 MFMA accumulators in VGPRs (gfx950's unified
    # register file); without it hipcc copies all 15 Gram tiles VGPR<->AGPR every k-step.
    cmd = [hipcc(), "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-mllvm", "-amdgpu-mfma-vgpr-form",
           "-I", os.path.join(ROOT, "include"), "-I", CSRC,
           os.path.join(CSRC, "gst.hip"), "-o", out + ".tmp"]
    if stamps:
        cmd.insert(4, "-DGST_STAMPS")
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    build(force="--force" in sys.argv, stamps="--stamps" in sys.argv)
