"""``kfp.v2`` surface: ``dsl``, ``compiler``, ``google.client``."""
from . import dsl, compiler, google  # noqa: F401
