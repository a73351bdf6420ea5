"""Artifact and I/O annotation types of the pipeline DSL.

Mirrors the kfp.v2.dsl type surface the reference imports (pytorch-pipeline.ipynb
cell 3, nb:50-51): ``Artifact, Dataset, Input, InputPath, Model, Output, OutputPath,
ClassificationMetrics, Metrics``.  Artifacts are plain objects holding a ``uri``, a local
``path`` (the orchestrator materialises every URI as a file path, as Vertex does with its
``/gcs/`` fuse mount) and a ``metadata`` dict that is round-tripped through the executor
output JSON.
"""
from __future__ import annotations

import json
import os
from typing import Any, Dict, Generic, List, Optional, TypeVar

__all__ = [
    "Artifact", "Dataset", "Model", "Metrics", "ClassificationMetrics",
    "SlicedClassificationMetrics", "HTML", "Markdown", "Input", "Output",
    "InputPath", "OutputPath", "ARTIFACT_TYPES", "artifact_class_for_schema",
]


class Artifact:
    """Generic artifact (schema ``system.Artifact``)."""

    schema_title = "system.Artifact"
    schema_version = "0.0.1"
    TYPE_NAME = "system.Artifact"

    def __init__(self, name: str = "", uri: str = "", metadata: Optional[Dict[str, Any]] = None):
        self.name = name
        self.uri = uri
        self.metadata: Dict[str, Any] = dict(metadata or {})

    # kfp resolves ``gs://`` URIs to the ``/gcs/`` fuse mount; mipipe resolves them into
    # the local object store root (mipipe.storage).
    @property
    def path(self) -> str:
        from mipipe.storage.gcs import uri_to_local_path
        return uri_to_local_path(self.uri)

    @path.setter
    def path(self, value: str) -> None:
        from mipipe.storage.gcs import local_path_to_uri
        self.uri = local_path_to_uri(value)

    def to_dict(self) -> Dict[str, Any]:
        return {"name": self.name, "uri": self.uri, "metadata": self.metadata,
                "type": {"schemaTitle": self.schema_title, "schemaVersion": self.schema_version}}

    def __repr__(self) -> str:
        return f"{type(self).__name__}(name={self.name!r}, uri={self.uri!r}, metadata={self.metadata!r})"


class Dataset(Artifact):
    schema_title = TYPE_NAME = "system.Dataset"


class Model(Artifact):
    schema_title = TYPE_NAME = "system.Model"

    @property
    def framework(self) -> str:
        return self.metadata.get("framework", "")

    @framework.setter
    def framework(self, v: str) -> None:
        self.metadata["framework"] = v


class Metrics(Artifact):
    """Scalar metrics (schema ``system.Metrics``); ``log_metric`` writes into metadata."""

    schema_title = TYPE_NAME = "system.Metrics"

    def log_metric(self, metric: str, value: float) -> None:
        self.metadata[metric] = value


class ClassificationMetrics(Artifact):
    schema_title = TYPE_NAME = "system.ClassificationMetrics"

    def log_roc_data_point(self, fpr: float, tpr: float, threshold: float) -> None:
        roc = self.metadata.setdefault("confidenceMetrics", [])
        roc.append({"confidenceThreshold": threshold, "recall": tpr, "falsePositiveRate": fpr})

    def log_roc_curve(self, fpr: List[float], tpr: List[float], threshold: List[float]) -> None:
        for f, t, th in zip(fpr, tpr, threshold):
            self.log_roc_data_point(f, t, th)

    def set_confusion_matrix_categories(self, categories: List[str]) -> None:
        self.metadata["confusionMatrix"] = {
            "annotationSpecs": [{"displayName": c} for c in categories],
            "rows": [{"row": [0] * len(categories)} for _ in categories],
        }

    def log_confusion_matrix_row(self, row_category: str, row: List[float]) -> None:
        cm = self.metadata["confusionMatrix"]
        names = [s["displayName"] for s in cm["annotationSpecs"]]
        cm["rows"][names.index(row_category)] = {"row": list(row)}

    def log_confusion_matrix(self, categories: List[str], matrix: List[List[float]]) -> None:
        self.set_confusion_matrix_categories(categories)
        for c, r in zip(categories, matrix):
            self.log_confusion_matrix_row(c, r)


class SlicedClassificationMetrics(Artifact):
    schema_title = TYPE_NAME = "system.SlicedClassificationMetrics"


class HTML(Artifact):
    schema_title = TYPE_NAME = "system.HTML"


class Markdown(Artifact):
    schema_title = TYPE_NAME = "system.Markdown"


ARTIFACT_TYPES = {c.schema_title: c for c in
                  (Artifact, Dataset, Model, Metrics, ClassificationMetrics,
                   SlicedClassificationMetrics, HTML, Markdown)}


def artifact_class_for_schema(schema_title: str):
    return ARTIFACT_TYPES.get(schema_title, Artifact)


T = TypeVar("T")


class _IOMarker:
    direction = ""

    def __init__(self, artifact_type=None):
        self.artifact_type = artifact_type


class _InputMeta(type):
    def __getitem__(cls, item):
        return _InputAnnotation(item)


class _OutputMeta(type):
    def __getitem__(cls, item):
        return _OutputAnnotation(item)


class _InputAnnotation(_IOMarker):
    direction = "input"


class _OutputAnnotation(_IOMarker):
    direction = "output"


class Input(metaclass=_InputMeta):
    """``Input[Dataset]``: the component receives an artifact object."""


class Output(metaclass=_OutputMeta):
    """``Output[Model]``: the component receives an artifact object to fill."""


class InputPath(_IOMarker):
    """``InputPath()``: the component receives a local file path of an input artifact.

    A ``_path``/``_file`` suffix of the argument name is stripped in the IR (kfp
    convention): ``input_file_path`` -> ``input_file``.
    """

    direction = "input_path"

    def __init__(self, type=None):  # noqa: A002 - kfp's keyword
        super().__init__(type)


class OutputPath(_IOMarker):
    """``OutputPath()``: the component receives a local path to write an output artifact."""

    direction = "output_path"

    def __init__(self, type=None):  # noqa: A002
        super().__init__(type)


def schema_for(artifact_type) -> str:
    """Schema title for an annotation's artifact type (class, string or None)."""
    if artifact_type is None:
        return Artifact.schema_title
    if isinstance(artifact_type, str):
        key = artifact_type if artifact_type.startswith("system.") else "system." + artifact_type
        return key if key in ARTIFACT_TYPES else Artifact.schema_title
    if isinstance(artifact_type, type) and issubclass(artifact_type, Artifact):
        return artifact_type.schema_title
    return Artifact.schema_title


def write_json(path: str, obj: Any) -> None:
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        json.dump(obj, f, indent=2, sort_keys=True)
    os.replace(tmp, path)
