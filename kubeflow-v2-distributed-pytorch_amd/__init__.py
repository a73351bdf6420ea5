"""mipipe — MI355X-native Kubeflow-v2-style pipelines + distributed training.

Import is cheap: subpackages are loaded lazily so that the pipeline DSL/compiler can be
used on machines without a GPU (or without torch initialised).
"""
__version__ = "0.1.0"
