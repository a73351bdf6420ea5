"""DSL -> kfp v2 pipeline-spec JSON (``from mipipe.compiler import Compiler``)."""
from .compiler import Compiler, compile_pipeline, component_to_yaml, SCHEMA_VERSION  # noqa: F401
