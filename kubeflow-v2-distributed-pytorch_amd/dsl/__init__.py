"""Pipeline DSL — the kfp.v2.dsl surface the reference uses (nb:46-53).

    from mipipe.dsl import component, pipeline, InputPath, OutputPath, Input, Output, \
        Artifact, Dataset, Model, Metrics, ClassificationMetrics, Condition, importer
"""
from .types import (Artifact, ClassificationMetrics, Dataset, HTML, Input, InputPath,  # noqa: F401
                    Markdown, Metrics, Model, Output, OutputPath, SlicedClassificationMetrics)
from .component import Component, component  # noqa: F401
from .pipeline import (Condition, ExitHandler, Pipeline, PipelineParam, PipelineTask,  # noqa: F401
                       TaskOutput, importer, pipeline)

__all__ = ["Artifact", "ClassificationMetrics", "Dataset", "HTML", "Input", "InputPath",
           "Markdown", "Metrics", "Model", "Output", "OutputPath",
           "SlicedClassificationMetrics", "Component", "component", "Condition",
           "ExitHandler", "Pipeline", "PipelineParam", "PipelineTask", "TaskOutput",
           "importer", "pipeline"]
