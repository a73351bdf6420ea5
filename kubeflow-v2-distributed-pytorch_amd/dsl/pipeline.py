"""``@pipeline``, tasks, channels and control flow of the DSL.

Reference: ``@kfp.dsl.pipeline(name="download-file"+uuid4)`` over
``def pipeline(baseline_accuracy: float = 70.0)`` whose body calls
``download_file('test-pkl','task.py')`` then ``train(download_file_task.output)``
(pytorch-pipeline.ipynb nb:218-221).  Calling a component inside the pipeline function
returns a :class:`PipelineTask`; ``task.output`` / ``task.outputs[name]`` are
:class:`TaskOutput` channels that the compiler turns into ``taskOutputArtifact`` /
``taskOutputParameter`` references.  :class:`Condition` gates a group of tasks on a
comparison (used to wire the reference's unused ``baseline_accuracy`` into an eval gate,
SURVEY §5.9).
"""
from __future__ import annotations

import contextlib
import inspect
import threading
from typing import Any, Callable, Dict, List, Optional

from .component import Component, sanitize_name

__all__ = ["pipeline", "Pipeline", "PipelineParam", "TaskOutput", "PipelineTask",
           "Condition", "ExitHandler", "importer", "current_builder", "ConditionOperator"]

_local = threading.local()


def current_builder() -> Optional["PipelineBuilder"]:
    stack = getattr(_local, "builders", None)
    return stack[-1] if stack else None


class _Channel:
    """Something that can feed a task input: pipeline param or upstream output."""

    def _cmp(self, op: str, other) -> "ConditionOperator":
        return ConditionOperator(op, self, other)

    def __eq__(self, other):  # type: ignore[override]
        return self._cmp("==", other)

    def __ne__(self, other):  # type: ignore[override]
        return self._cmp("!=", other)

    def __lt__(self, other):
        return self._cmp("<", other)

    def __le__(self, other):
        return self._cmp("<=", other)

    def __gt__(self, other):
        return self._cmp(">", other)

    def __ge__(self, other):
        return self._cmp(">=", other)

    __hash__ = object.__hash__


class PipelineParam(_Channel):
    """A pipeline input parameter (``baseline_accuracy: float = 70.0``, nb:219)."""

    def __init__(self, name: str, param_type: str, default: Any = inspect.Parameter.empty):
        self.name = name
        self.param_type = param_type
        self.default = default

    @property
    def pattern(self) -> str:
        return f"{{{{pipelineparam:op=;name={self.name}}}}}"

    def __repr__(self) -> str:
        return f"PipelineParam({self.name!r})"


class TaskOutput(_Channel):
    def __init__(self, task: "PipelineTask", name: str, kind: str, type_: str):
        self.task = task
        self.name = name
        self.kind = kind      # 'parameter' | 'artifact'
        self.type = type_

    def __repr__(self) -> str:
        return f"TaskOutput({self.task.name}.{self.name})"


class ConditionOperator:
    def __init__(self, op: str, lhs, rhs):
        self.op, self.lhs, self.rhs = op, lhs, rhs


class _Outputs(dict):
    def __init__(self, task):
        super().__init__()
        self._task = task

    def __missing__(self, key):
        raise KeyError(f"task {self._task.name!r} has no output {key!r}; "
                       f"outputs: {sorted(self)}")


class PipelineTask:
    """One component invocation inside a pipeline."""

    def __init__(self, comp: Component, arguments: Dict[str, Any], builder: "PipelineBuilder"):
        self.component = comp
        self.arguments = arguments
        self.builder = builder
        self.name = builder.unique_task_name(comp.name)
        self.display_name: Optional[str] = None
        self.dependent_tasks: List[str] = []
        self.enable_caching = True
        self.retries = 0
        self.env: Dict[str, str] = {}
        self.resources: Dict[str, Any] = {}
        self.group = builder.current_group()
        self.outputs = _Outputs(self)
        for spec in comp.outputs:
            self.outputs[spec.name] = TaskOutput(self, spec.name, spec.kind, spec.type)
        for v in arguments.values():
            if isinstance(v, TaskOutput) and v.task.name not in self.dependent_tasks:
                self.dependent_tasks.append(v.task.name)
        builder.add_task(self)

    @property
    def output(self) -> TaskOutput:
        if len(self.outputs) != 1:
            raise AttributeError(
                f"task {self.name!r} has {len(self.outputs)} outputs; use .outputs[name]")
        return next(iter(self.outputs.values()))

    # kfp-style fluent setters ------------------------------------------------
    def after(self, *tasks: "PipelineTask") -> "PipelineTask":
        for t in tasks:
            if t.name not in self.dependent_tasks:
                self.dependent_tasks.append(t.name)
        return self

    def set_display_name(self, name: str) -> "PipelineTask":
        self.display_name = name
        return self

    def set_caching_options(self, enable_caching: bool) -> "PipelineTask":
        self.enable_caching = bool(enable_caching)
        return self

    def set_retry(self, num_retries: int, backoff_duration: Optional[str] = None,
                  backoff_factor: Optional[float] = None,
                  backoff_max_duration: Optional[str] = None) -> "PipelineTask":
        self.retries = int(num_retries)
        return self

    def set_env_variable(self, name: str, value: str) -> "PipelineTask":
        self.env[name] = str(value)
        return self

    def set_cpu_limit(self, cpu: str) -> "PipelineTask":
        self.resources["cpuLimit"] = cpu
        return self

    def set_memory_limit(self, memory: str) -> "PipelineTask":
        self.resources["memoryLimit"] = memory
        return self

    def set_gpu_limit(self, gpu) -> "PipelineTask":
        self.resources["accelerator"] = {"type": "AMD_INSTINCT_MI355X", "count": int(gpu)}
        return self

    set_accelerator_limit = set_gpu_limit

    def __repr__(self) -> str:
        return f"PipelineTask({self.name!r})"


class _Group:
    def __init__(self, kind: str, name: str, parent: Optional["_Group"], condition=None):
        self.kind = kind          # 'root' | 'condition' | 'exit_handler'
        self.name = name
        self.parent = parent
        self.condition = condition
        self.tasks: List[PipelineTask] = []
        self.groups: List["_Group"] = []
        self.exit_task: Optional[PipelineTask] = None

    def all_tasks(self) -> List[PipelineTask]:
        out = list(self.tasks)
        for g in self.groups:
            out.extend(g.all_tasks())
        return out


class PipelineBuilder:
    def __init__(self, name: str):
        self.name = name
        self.tasks: Dict[str, PipelineTask] = {}
        self.root = _Group("root", "root", None)
        self._group_stack = [self.root]
        self._counters: Dict[str, int] = {}

    def unique_task_name(self, base: str) -> str:
        n = self._counters.get(base, 0) + 1
        self._counters[base] = n
        return base if n == 1 else f"{base}-{n}"

    def group_name(self, base: str) -> str:
        n = self._counters.get("#" + base, 0) + 1
        self._counters["#" + base] = n
        return f"{base}-{n}"

    def current_group(self) -> _Group:
        return self._group_stack[-1]

    def add_task(self, t: PipelineTask) -> None:
        self.tasks[t.name] = t
        self.current_group().tasks.append(t)

    def push_group(self, g: _Group) -> None:
        self.current_group().groups.append(g)
        self._group_stack.append(g)

    def pop_group(self) -> None:
        self._group_stack.pop()


class Condition:
    """``with Condition(train.outputs['accuracy'] >= baseline_accuracy):`` — tasks inside run
    only when the comparison holds (kfp ``dsl.Condition``; compiled to a sub-DAG with a
    ``triggerPolicy.condition``)."""

    def __init__(self, condition: ConditionOperator, name: Optional[str] = None):
        if not isinstance(condition, ConditionOperator):
            raise TypeError("Condition expects a comparison of a pipeline channel")
        self.condition = condition
        self.name = name
        self._group: Optional[_Group] = None

    def __enter__(self):
        b = current_builder()
        if b is None:
            raise RuntimeError("Condition used outside a pipeline")
        self._group = _Group("condition", b.group_name("condition"), b.current_group(),
                             condition=self.condition)
        b.push_group(self._group)
        return self

    def __exit__(self, *exc):
        current_builder().pop_group()
        return False


class ExitHandler:
    """``with ExitHandler(exit_task):`` — ``exit_task`` runs after the group, even on failure."""

    def __init__(self, exit_task: PipelineTask, name: Optional[str] = None):
        self.exit_task = exit_task
        self.name = name

    def __enter__(self):
        b = current_builder()
        g = _Group("exit_handler", b.group_name("exit-handler"), b.current_group())
        g.exit_task = self.exit_task
        # the exit task was created before the group: move it out of the parent's task list
        # is not needed — it stays at the parent level and depends on the whole group.
        self._group = g
        b.push_group(g)
        return self

    def __exit__(self, *exc):
        current_builder().pop_group()
        return False


_IMPORTER_COUNTER = [0]


def importer(artifact_uri, artifact_class=None, reimport: bool = False,
             metadata: Optional[dict] = None) -> PipelineTask:
    """Import an existing object (``gs://...``) as an artifact — what the reference's
    placeholder cell ``#importer to get the task.py file to the second component``
    (nb:10) intended instead of the download step."""
    from .types import Artifact
    from .component import Component
    cls = artifact_class or Artifact
    schema = cls.schema_title

    def importer_fn(uri: str, artifact=None):
        raise RuntimeError("importer runs inside the orchestrator")

    comp = Component.__new__(Component)
    comp.python_func = importer_fn
    comp.function_name = "importer"
    comp.name = "importer"
    comp.description = "artifact importer"
    comp.base_image = ""
    comp.packages_to_install = []
    comp.pip_index_urls = []
    from .component import IOSpec
    comp.inputs = [IOSpec("uri", "uri", "parameter", "STRING", "value")]
    comp.outputs = [IOSpec("artifact", "artifact", "artifact", schema, "path")]
    comp.source = ""
    comp.is_importer = True
    comp.importer_spec = {"reimport": bool(reimport), "metadata": dict(metadata or {}),
                          "typeSchema": {"schemaTitle": schema}}
    b = current_builder()
    if b is None:
        raise RuntimeError("importer used outside a pipeline")
    return PipelineTask(comp, {"uri": artifact_uri}, b)


class Pipeline:
    """Result of ``@pipeline``: holds the function and its metadata; callable like it."""

    def __init__(self, func: Callable, name: Optional[str], description: Optional[str],
                 pipeline_root: Optional[str]):
        self.pipeline_func = func
        self.name = name or sanitize_name(func.__name__)
        self.description = description or (inspect.getdoc(func) or "")
        self.pipeline_root = pipeline_root
        self.__name__ = func.__name__
        self.__doc__ = func.__doc__
        self.__wrapped__ = func
        # kfp stores these attributes on the function object
        self._component_human_name = self.name

    def parameters(self) -> List[PipelineParam]:
        from .component import _param_type
        sig = inspect.signature(self.pipeline_func)
        out = []
        for p in sig.parameters.values():
            ann = p.annotation
            if isinstance(ann, str):
                ann = {"str": str, "int": int, "float": float, "bool": bool}.get(ann, str)
            out.append(PipelineParam(p.name, _param_type(ann), p.default))
        return out

    def build(self) -> PipelineBuilder:
        b = PipelineBuilder(self.name)
        params = self.parameters()
        stack = getattr(_local, "builders", None)
        if stack is None:
            stack = _local.builders = []
        stack.append(b)
        try:
            self.pipeline_func(*params)
        finally:
            stack.pop()
        b.params = params
        return b

    def __call__(self, *args, **kwargs):
        # nested pipelines are not supported; calling outside compilation runs the body
        # in a builder (useful for inspection)
        return self.pipeline_func(*args, **kwargs)


def pipeline(func: Optional[Callable] = None, *, name: Optional[str] = None,
             description: Optional[str] = None, pipeline_root: Optional[str] = None):
    def wrap(f):
        return Pipeline(f, name, description, pipeline_root)

    if func is not None:
        return wrap(func)
    return wrap
