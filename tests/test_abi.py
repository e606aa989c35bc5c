"""CPU-side checks of the C ABI: the library loads and exports every declared symbol."""
import ctypes as ct
import os
import re

import numpy as np
import pytest

from gibbs_student_t_amd import _abi
from gibbs_student_t_amd.native import model_desc
from golden_io import load_ref

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "gst.h")


def declared_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^int\s+(gst_\w+)\s*\(", src, flags=re.M)))


def test_header_and_binding_agree():
    assert set(declared_functions()) == set(_abi.EXPORTS)


@pytest.mark.skipif(not os.path.exists(_abi.LIB_PATH), reason="libgst.so not built")
def test_library_exports_every_declared_symbol():
    lib = ct.CDLL(_abi.LIB_PATH)
    for name in declared_functions():
        assert hasattr(lib, name), name
    lib2 = _abi.load()
    assert lib2.gst_version() == _abi.ABI_VERSION
    assert lib2.gst_tape_stride(130, 74) == 120 + 74 + 2 + 2 * 130


@pytest.mark.skipif(not os.path.exists(_abi.LIB_PATH), reason="libgst.so not built")
def test_error_path_without_gpu_is_loud():
    """No device here: creating a context must fail with a message, not crash."""
    lib = _abi.load()
    ctx = ct.c_void_p()
    rc = lib.gst_ctx_create(0, ct.byref(ctx))
    if rc == 0:  # running on a GPU box
        lib.gst_ctx_destroy(ctx)
        pytest.skip("a device is present")
    assert rc < 0 and _abi.last_error(lib)


def test_model_desc_packing():
    ref = load_ref("beta_efac_fixed")
    desc, keep = model_desc(ref["pta"], ref["kw"])
    assert (desc.n, desc.m, desc.nfourier, desc.ntm, desc.nparams) == (130, 74, 60, 14, 4)
    names = ref["pta"].param_names
    assert names[desc.idx_efac].endswith("efac")
    assert names[desc.idx_gamma].endswith("gamma")
    assert desc.n_hyper == 2 and desc.n_white == 2
    assert desc.model == _abi.GST_MODEL_MIXTURE and desc.theta_prior_beta == 1
    T = np.ctypeslib.as_array(desc.T, shape=(desc.n * desc.m,)).reshape(desc.n, desc.m)
    np.testing.assert_array_equal(T, ref["pta"].T)


def test_missing_library_raises(tmp_path):
    with pytest.raises(_abi.GstNativeError):
        _abi.load(str(tmp_path / "nope.so"))


def test_header_is_valid_c():
    """include/gst.h compiles as C on its own (a C / cgo / ctypes consumer includes it bare)."""
    import shutil
    import subprocess
    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        pytest.skip("no C compiler")
    hdr = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include",
                       "gst.h")
    r = subprocess.run([cc, "-fsyntax-only", "-Wall", "-Werror", "-x", "c", hdr],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
