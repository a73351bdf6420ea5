"""Local ``gs://`` object store and Google-Cloud client aliases (see :mod:`mipipe.storage.gcs`)."""
from __future__ import annotations

import importlib
import sys
import types

from . import gcs  # noqa: F401
from .gcs import Blob, Bucket, Client, gcs_root, uri_to_local_path, local_path_to_uri  # noqa: F401


def _module_importable(name: str) -> bool:
    try:
        importlib.import_module(name)
        return True
    except Exception:
        return False


def install_google_cloud_alias(force: bool = False) -> None:
    """Make ``from google.cloud import storage, aiplatform`` resolve to mipipe's local
    implementations when the real Google client libraries are absent (no network on the
    MI355X node).  Lets the reference's component bodies (nb:101-106, nb:127-196) and
    task.py's model export (task.py:19, 286-294) run unmodified.
    """
    if not force and _module_importable("google.cloud.storage"):
        return
    from mipipe import aiplatform as _aip

    google = sys.modules.get("google") or types.ModuleType("google")
    if not hasattr(google, "__path__"):
        google.__path__ = []  # namespace-like
    cloud = sys.modules.get("google.cloud") or types.ModuleType("google.cloud")
    if not hasattr(cloud, "__path__"):
        cloud.__path__ = []
    cloud.storage = gcs
    cloud.aiplatform = _aip
    google.cloud = cloud
    sys.modules["google"] = google
    sys.modules["google.cloud"] = cloud
    sys.modules["google.cloud.storage"] = gcs
    sys.modules["google.cloud.aiplatform"] = _aip
    sys.modules["google.cloud.aiplatform.gapic"] = _aip.gapic
