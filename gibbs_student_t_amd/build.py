"""Build libgst.so in-tree with hipcc for gfx950 (no JIT cache: the .so travels with the repo)."""
from __future__ import annotations

import os
import re
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libgst.so")
SOURCES = [os.path.join(CSRC, f) for f in ("gst.hip", "gst_inst.hip", "gst_shapes.h", "gst_sim.hpp",
                                            "gst_kernel.hpp", "gst_large.hpp", "philox.hpp")]
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


def shapes():
    """The persistent kernel's shapes, from the GST_SHAPES list in csrc/gst_shapes.h."""
    txt = open(os.path.join(CSRC, "gst_shapes.h")).read()
    body = txt[txt.index("#define GST_SHAPES(X)"):txt.index("#define GST_PICK_NAME")]
    return re.findall(r"X\((\d+), (\d+), (\d+), (\d+), (\d)\)", body)


def build(force: bool = False, verbose: bool = True, stamps: bool = False,
          jobs: int | None = None) -> str:
    """Compile libgst.so (or the diagnostic libgst_stamps.so with per-stage cycle stamps):
    gst.hip (ABI, large path) and one gst_inst.hip object per persistent-kernel shape,
    compiled in parallel, linked into one shared library."""
    # experimental variants (not the product library): GST_BUILD_VARIANT=name builds
    # libgst_<name>.so with GST_EXTRA_CFLAGS added, for A/B timing via GST_LIB
    variant = os.environ.get("GST_BUILD_VARIANT", "")
    out = STAMPS_LIB if stamps else (os.path.join(HERE, f"libgst_{variant}.so") if variant else LIB)
    if not force and not stamps and not variant and up_to_date():
        return LIB
    objdir = os.path.join(HERE, "_obj_stamps" if stamps else (f"_obj_{variant}" if variant else "_obj"))
    os.makedirs(objdir, exist_ok=True)
    # -amdgpu-mfma-vgpr-form: keep the fp64 MFMA accumulators in VGPRs (gfx950's unified
    # register file); without it hipcc copies all 15 Gram tiles VGPR<->AGPR every k-step.
    # -disable-machine-licm: the sweep loop body is one huge block; MachineLICM hoists every
    # loop-invariant fp64 constant (polynomial coefficients of log/exp/cos, ...) and lane
    # address out of it into VGPRs, and at 256 registers (two chains per SIMD) the allocator
    # then spills them and reloads them from scratch inside the rejection / MH loops.
    # Rematerialised in place they cost SALU moves: 576 -> 320 B/lane spill, +7.8% sweeps/s
    # at 2048 chains.
    base = [hipcc(), "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
            "-mllvm", "-amdgpu-mfma-vgpr-form", "-mllvm", "-disable-machine-licm",
            "-I", os.path.join(ROOT, "include"), "-I", CSRC]
    if stamps:
        base.append("-DGST_STAMPS")
    base += os.environ.get("GST_EXTRA_CFLAGS", "").split()
    units = [(os.path.join(CSRC, "gst.hip"), [], os.path.join(objdir, "gst.o"))]
    for sh in shapes():
        units.append((os.path.join(CSRC, "gst_inst.hip"), ["-DGST_SHAPE=" + ",".join(sh)],
                      os.path.join(objdir, "inst_" + "_".join(sh) + ".o")))

    # incremental (not for force=True): a unit is recompiled when its object is missing, older
    # than one of its sources, or was built with other flags (a .cmd file beside it)
    kern_deps = [os.path.join(CSRC, f) for f in ("gst_kernel.hpp", "philox.hpp", "gst_shapes.h")]
    deps = {"gst.hip": SOURCES + [HEADER],
            "gst_inst.hip": kern_deps + [os.path.join(CSRC, "gst_inst.hip"), HEADER]}

    def compile_one(u):
        src, extra, obj = u
        cmd = base + extra + ["-c", src, "-o", obj]
        stamp = obj + ".cmd"
        if not force and os.path.exists(obj) and os.path.exists(stamp) and \
                open(stamp).read() == " ".join(cmd) and \
                all(os.path.getmtime(d) <= os.path.getmtime(obj)
                    for d in deps[os.path.basename(src)]):
            return obj
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        with open(stamp, "w") as f:
            f.write(" ".join(cmd))
        return obj

    jobs = jobs or int(os.environ.get("MAX_JOBS", 0)) or min(8, os.cpu_count() or 1)
    with ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(compile_one, units))
    cmd = [hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC"] + objs + ["-o", out + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    build(force="--force" in sys.argv, stamps="--stamps" in sys.argv)
