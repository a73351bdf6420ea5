"""``kfp.v2.google`` surface."""
from . import client  # noqa: F401
