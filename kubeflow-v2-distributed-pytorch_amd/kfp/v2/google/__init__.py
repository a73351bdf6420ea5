"""``kfp.v2.google.client`` surface."""
from mipipe import client  # noqa: F401
