"""Local object store with ``gs://`` URIs (replaces Google Cloud Storage).

The reference talks to GCS in three places: the ``download_file`` component
(pytorch-pipeline.ipynb nb:101-106: ``storage.Client().bucket(b).blob(k)
.download_to_filename(p)``), the model export in task.py (task.py:286-294:
``storage.blob.Blob.from_string(uri, client=storage.Client()).upload_from_filename``)
and Vertex's staging / pipeline_root buckets.  On one MI355X node with no network those
become a directory tree: ``gs://bucket/key`` <-> ``$MIPIPE_GCS_ROOT/bucket/key``.

The API mirrors the subset of ``google.cloud.storage`` the reference uses, so unmodified
component code runs once :func:`mipipe.storage.install_google_cloud_alias` has mapped
``google.cloud.storage`` onto this module.  The ``/gcs/<bucket>/<key>`` fuse-style path
that Vertex exposes inside containers is accepted everywhere a path is.
"""
from __future__ import annotations

import os
import shutil
from typing import Iterator, List, Optional, Tuple

__all__ = ["Client", "Bucket", "Blob", "gcs_root", "parse_gs_uri", "uri_to_local_path",
           "local_path_to_uri", "blob"]


def gcs_root() -> str:
    root = os.environ.get("MIPIPE_GCS_ROOT")
    if not root:
        root = os.path.join(os.path.expanduser("~"), ".mipipe", "gcs")
    return os.path.abspath(root)


def parse_gs_uri(uri: str) -> Tuple[str, str]:
    if uri.startswith("gs://"):
        rest = uri[5:]
    elif uri.startswith("/gcs/"):
        rest = uri[5:]
    else:
        raise ValueError(f"not a gs:// URI: {uri!r}")
    bucket, _, key = rest.partition("/")
    if not bucket:
        raise ValueError(f"URI has no bucket: {uri!r}")
    return bucket, key


def uri_to_local_path(uri: str) -> str:
    """Map ``gs://b/k`` / ``/gcs/b/k`` / ``file://p`` / plain path to a local path."""
    if not uri:
        return ""
    if uri.startswith("gs://") or uri.startswith("/gcs/"):
        b, k = parse_gs_uri(uri)
        return os.path.join(gcs_root(), b, k)
    if uri.startswith("file://"):
        return uri[7:]
    return uri


def local_path_to_uri(path: str) -> str:
    """Inverse of :func:`uri_to_local_path` for paths under the store root."""
    ap = os.path.abspath(path)
    root = gcs_root()
    if ap.startswith(root + os.sep):
        return "gs://" + os.path.relpath(ap, root).replace(os.sep, "/")
    return ap


class Blob:
    def __init__(self, name: str, bucket: "Bucket"):
        self.name = name
        self.bucket = bucket

    @classmethod
    def from_string(cls, uri: str, client: Optional["Client"] = None) -> "Blob":
        b, k = parse_gs_uri(uri)
        return cls(k, Bucket(client or Client(), b))

    @property
    def local_path(self) -> str:
        return os.path.join(self.bucket.local_path, self.name)

    @property
    def public_url(self) -> str:
        return f"gs://{self.bucket.name}/{self.name}"

    def exists(self, client=None) -> bool:
        return os.path.isfile(self.local_path)

    @property
    def size(self) -> Optional[int]:
        return os.path.getsize(self.local_path) if self.exists() else None

    def download_to_filename(self, filename: str, client=None) -> None:
        if not self.exists():
            raise FileNotFoundError(f"No such object: {self.public_url}")
        d = os.path.dirname(os.path.abspath(filename))
        os.makedirs(d, exist_ok=True)
        shutil.copyfile(self.local_path, filename)

    def download_as_bytes(self, client=None) -> bytes:
        if not self.exists():
            raise FileNotFoundError(f"No such object: {self.public_url}")
        with open(self.local_path, "rb") as f:
            return f.read()

    def download_as_string(self, client=None) -> bytes:
        return self.download_as_bytes()

    def download_as_text(self, client=None, encoding: str = "utf-8") -> str:
        return self.download_as_bytes().decode(encoding)

    def _atomic_write(self, writer) -> None:
        os.makedirs(os.path.dirname(self.local_path), exist_ok=True)
        tmp = f"{self.local_path}.tmp.{os.getpid()}"
        writer(tmp)
        os.replace(tmp, self.local_path)

    def upload_from_filename(self, filename: str, content_type=None, client=None) -> None:
        self._atomic_write(lambda tmp: shutil.copyfile(filename, tmp))

    def upload_from_string(self, data, content_type=None, client=None) -> None:
        if isinstance(data, str):
            data = data.encode("utf-8")

        def w(tmp):
            with open(tmp, "wb") as f:
                f.write(data)
        self._atomic_write(w)

    def delete(self, client=None) -> None:
        os.remove(self.local_path)


class Bucket:
    def __init__(self, client: "Client", name: str):
        self.client = client
        self.name = name

    @property
    def local_path(self) -> str:
        return os.path.join(gcs_root(), self.name)

    def blob(self, blob_name: str) -> Blob:
        return Blob(blob_name, self)

    def get_blob(self, blob_name: str) -> Optional[Blob]:
        b = Blob(blob_name, self)
        return b if b.exists() else None

    def exists(self) -> bool:
        return os.path.isdir(self.local_path)

    def list_blobs(self, prefix: str = "") -> Iterator[Blob]:
        return self.client.list_blobs(self, prefix=prefix)


class Client:
    def __init__(self, project: Optional[str] = None, credentials=None, **_):
        self.project = project

    def bucket(self, bucket_name: str) -> Bucket:
        return Bucket(self, bucket_name)

    def get_bucket(self, bucket_name: str) -> Bucket:
        b = Bucket(self, bucket_name)
        if not b.exists():
            raise FileNotFoundError(f"No such bucket: gs://{bucket_name}")
        return b

    def create_bucket(self, bucket_name: str, **_) -> Bucket:
        b = Bucket(self, bucket_name)
        os.makedirs(b.local_path, exist_ok=True)
        return b

    def list_blobs(self, bucket_or_name, prefix: str = "") -> Iterator[Blob]:
        b = bucket_or_name if isinstance(bucket_or_name, Bucket) else Bucket(self, bucket_or_name)
        out: List[Blob] = []
        for dirpath, _, files in os.walk(b.local_path):
            for fn in files:
                key = os.path.relpath(os.path.join(dirpath, fn), b.local_path).replace(os.sep, "/")
                if key.startswith(prefix) and ".tmp." not in key:
                    out.append(Blob(key, b))
        return iter(sorted(out, key=lambda x: x.name))


class _BlobModule:
    """``storage.blob.Blob`` access path used at task.py:293."""

    Blob = Blob


blob = _BlobModule()
