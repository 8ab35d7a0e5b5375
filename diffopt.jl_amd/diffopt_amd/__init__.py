"""diffopt_amd — MI355X-native sensitivity-solve engine for DiffOpt.jl's
QuadraticProgram and ConicProgram back-ends (host side; the compute is the HIP
library libdiffopt_mi355x.so behind include/diffopt_mi355x.h)."""

from . import _lib  # noqa: F401
from ._lib import EngineError, EngineUnavailable, SingularException  # noqa: F401

__all__ = ["QuadraticProgram", "ConicProgram", "synthetic", "parallel"]


def __getattr__(name):
    import importlib
    if name == "QuadraticProgram":
        return importlib.import_module(".qp", __name__)
    if name == "ConicProgram":
        return importlib.import_module(".conic", __name__)
    if name in ("synthetic", "parallel", "qp", "conic"):
        return importlib.import_module("." + name, __name__)
    raise AttributeError(name)
