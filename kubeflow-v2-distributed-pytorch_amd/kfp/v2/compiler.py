"""``kfp.v2.compiler`` -> :mod:`mipipe.compiler`."""
from mipipe.compiler import Compiler, compile_pipeline  # noqa: F401
