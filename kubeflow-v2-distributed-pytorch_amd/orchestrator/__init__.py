"""Local DAG orchestrator (replaces Vertex AI Pipelines): :class:`PipelineRunner`."""
from .runner import PipelineRunner, RunFailed, run_job_spec, TERMINAL_STATES  # noqa: F401
