"""``kfp.v2.google.client`` -> :mod:`mipipe.client`."""
from mipipe.client import AIPlatformClient, Client  # noqa: F401
