"""Pipeline submission client (replaces ``kfp.v2.google.client.AIPlatformClient``)."""
from .client import AIPlatformClient, Client, RunHandle  # noqa: F401
