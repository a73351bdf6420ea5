"""``kfp.v2`` surface: ``dsl``, ``compiler``, ``google.client``."""
from mipipe import dsl  # noqa: F401
from mipipe import compiler  # noqa: F401
from . import google  # noqa: F401
