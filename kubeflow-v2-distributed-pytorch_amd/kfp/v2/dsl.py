"""``kfp.v2.dsl`` -> :mod:`mipipe.dsl`."""
from mipipe.dsl import *  # noqa: F401,F403
from mipipe.dsl import __all__  # noqa: F401
