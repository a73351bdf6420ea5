"""kfp-compatible import surface, so the reference notebook's imports work unchanged::

    import kfp; from kfp import dsl; from kfp.v2 import compiler
    from kfp.v2.dsl import component, InputPath, OutputPath, ...
    from kfp.v2.google.client import AIPlatformClient

resolve (after :func:`install_alias`, or with ``mipipe.kfp`` imported directly) to mipipe's
DSL (:mod:`mipipe.dsl`), compiler (:mod:`mipipe.compiler`) and client (:mod:`mipipe.client`).
kfp itself is not installed on the MI355X node (no network).
"""
import sys

from mipipe import dsl  # noqa: F401
from mipipe import compiler  # noqa: F401
from . import v2  # noqa: F401

__version__ = "1.8.22+mipipe"


def install_alias(force: bool = False) -> None:
    """Register ``kfp``, ``kfp.dsl``, ``kfp.v2``... in ``sys.modules`` (only when the real
    kfp is absent, unless ``force``)."""
    if not force:
        try:
            import importlib
            importlib.import_module("kfp")
            if not getattr(sys.modules["kfp"], "__version__", "").endswith("+mipipe"):
                return
        except ImportError:
            pass
    me = sys.modules[__name__]
    sys.modules["kfp"] = me
    sys.modules["kfp.dsl"] = dsl
    sys.modules["kfp.compiler"] = compiler
    sys.modules["kfp.v2"] = v2
    sys.modules["kfp.v2.dsl"] = v2.dsl
    sys.modules["kfp.v2.compiler"] = v2.compiler
    sys.modules["kfp.v2.google"] = v2.google
    sys.modules["kfp.v2.google.client"] = v2.google.client
    sys.modules["kfp.dsl"] = dsl
