"""MI355X-native batched Gibbs sampler for the Gaussian / Student-t / outlier-mixture
pulsar-timing noise model of aniwl/gibbs_student_t (reference gibbs.py).

``Gibbs`` is the drop-in sampler (GPU only, via libgst.so); ``model.PTA`` is the
structured noise model it consumes; ``data`` builds J1713+0747 and simulate_data-style
datasets.
"""
from . import model  # noqa: F401

__all__ = ["Gibbs", "model", "data", "build"]


def __getattr__(name):
    import importlib
    if name == "Gibbs":
        return importlib.import_module(__name__ + ".sampler").Gibbs
    if name in ("data", "build", "native", "sampler", "diag", "dist"):
        return importlib.import_module(__name__ + "." + name)
    raise AttributeError(name)
