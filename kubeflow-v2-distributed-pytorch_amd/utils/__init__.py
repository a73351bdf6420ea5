"""Driver-side configuration helpers.

The reference notebook loads a ``.env`` file with the python-dotenv IPython magic
(pytorch-pipeline.ipynb:74-75), reads ``PROJECT_ID`` / ``BUCKET`` from the environment and
derives ``PIPELINE_ROOT = gs://<BUCKET>/pipeline_root`` with a hard-coded region (nb:78-86).
python-dotenv is not installed here, so :func:`load_dotenv` parses the same file format itself:
``KEY=VALUE`` lines, optional ``export`` prefix, single / double quotes (double quotes honour
``\\n`` escapes), ``#`` comments and ``${VAR}`` expansion.
"""
from __future__ import annotations

import os
import re
from dataclasses import dataclass
from typing import Dict, Mapping, MutableMapping, Optional

__all__ = ["parse_dotenv", "load_dotenv", "PipelineConfig", "pipeline_config"]

_LINE = re.compile(r"^\s*(?:export\s+)?([A-Za-z_][A-Za-z0-9_.]*)\s*=\s*(.*)$")
_VAR = re.compile(r"\$\{([A-Za-z_][A-Za-z0-9_]*)\}")


def _unquote(raw: str) -> tuple:
    """-> (value, expand): quoted values end at the closing quote; unquoted ones at ' #'."""
    raw = raw.strip()
    if raw[:1] in ("'", '"'):
        q = raw[0]
        end = raw.find(q, 1)
        while q == '"' and end > 0 and raw[end - 1] == "\\":
            end = raw.find(q, end + 1)
        body = raw[1:end] if end > 0 else raw[1:]
        if q == '"':
            body = body.replace("\\n", "\n").replace('\\"', '"')
        return body, q == '"'
    hash_at = re.search(r"\s#", raw)
    return (raw[:hash_at.start()] if hash_at else raw).strip(), True


def parse_dotenv(text: str, env: Optional[Mapping[str, str]] = None) -> Dict[str, str]:
    """Parse ``.env`` text; ``${VAR}`` resolves against earlier keys, then ``env``."""
    env = os.environ if env is None else env
    out: Dict[str, str] = {}
    for line in text.splitlines():
        if not line.strip() or line.lstrip().startswith("#"):
            continue
        m = _LINE.match(line)
        if not m:
            continue
        value, expand = _unquote(m.group(2))
        if expand:
            value = _VAR.sub(lambda v: out.get(v.group(1), env.get(v.group(1), "")), value)
        out[m.group(1)] = value
    return out


def load_dotenv(path: str = ".env", override: bool = False,
                environ: Optional[MutableMapping[str, str]] = None) -> Dict[str, str]:
    """python-dotenv's ``load_dotenv``: export the file's variables into ``environ`` (existing
    variables win unless ``override``).  A missing file is not an error.  Returns the parsed
    values."""
    environ = os.environ if environ is None else environ
    if not os.path.isfile(path):
        return {}
    with open(path, encoding="utf-8") as f:
        values = parse_dotenv(f.read(), environ)
    for k, v in values.items():
        if override or k not in environ:
            environ[k] = v
    return values


@dataclass
class PipelineConfig:
    project_id: str
    bucket: str
    region: str
    pipeline_root: str


def pipeline_config(env: Optional[Mapping[str, str]] = None, region: str = "us-central1",
                    default_project: str = "local", default_bucket: str = "test-pkl") -> PipelineConfig:
    """The notebook's driver config (nb:78-86): PROJECT_ID / BUCKET from the environment,
    ``PIPELINE_ROOT = gs://<bucket>/pipeline_root`` (``gs://`` resolves to the local object
    store), region ``us-central1`` unless ``REGION`` is set."""
    env = os.environ if env is None else env
    project = env.get("PROJECT_ID", default_project)
    bucket = env.get("BUCKET", default_bucket)
    root = env.get("PIPELINE_ROOT", f"gs://{bucket}/pipeline_root")
    return PipelineConfig(project, bucket, env.get("REGION", region), root)
