"""``@component`` — lightweight Python components (kfp.v2 ``component`` equivalent).

Reference usage: ``@component(packages_to_install=["google-cloud-storage"])`` on
``download_file`` (pytorch-pipeline.ipynb nb:97-98) and on ``train`` (nb:122-123).
The decorator captures the function's source and signature; the body never runs at
definition time.  Inside a ``@pipeline`` function, calling the component records a
:class:`~mipipe.dsl.pipeline.PipelineTask`; the compiler turns the recorded graph into
the kfp v2 pipeline-spec JSON and the local orchestrator runs each task in its own
process through :mod:`mipipe.dsl.executor_main`.
"""
from __future__ import annotations

import inspect
import json
import re
import textwrap
import typing
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional

from . import types as T

__all__ = ["component", "Component", "IOSpec", "sanitize_name", "io_name_for_path_arg",
           "PARAMETER_TYPES", "DEFAULT_BASE_IMAGE"]

DEFAULT_BASE_IMAGE = "python:3.7"  # pipeline.png: both steps ran in python:3.7

# kfp 1.8 v2-compatible IR parameter types.  bool/dict/list travel as JSON strings.
PARAMETER_TYPES = {str: "STRING", int: "INT", float: "DOUBLE", bool: "STRING",
                   dict: "STRING", list: "STRING"}


def sanitize_name(name: str) -> str:
    """kfp naming: lower-case, ``[^a-z0-9]`` runs -> ``-`` (``download_file`` -> ``download-file``)."""
    return re.sub(r"-+", "-", re.sub(r"[^-0-9a-z]+", "-", name.lower())).strip("-")


def io_name_for_path_arg(arg_name: str) -> str:
    """``InputPath``/``OutputPath`` argument naming rule: strip one ``_path``
    suffix, else one ``_file`` suffix: ``output_file_path`` -> ``output_file``."""
    if arg_name.endswith("_path"):
        return arg_name[: -len("_path")]
    if arg_name.endswith("_file"):
        return arg_name[: -len("_file")]
    return arg_name


@dataclass
class IOSpec:
    name: str            # IR name
    py_name: str         # python argument name ('' for return outputs)
    kind: str            # 'parameter' | 'artifact'
    type: str            # IR parameter type or artifact schema title
    passing: str         # 'value' | 'path' | 'object' | 'return'
    default: Any = inspect.Parameter.empty
    py_type: Any = None

    @property
    def optional(self) -> bool:
        return self.default is not inspect.Parameter.empty


def _strip_optional(ann):
    origin = typing.get_origin(ann)
    if origin is typing.Union:
        args = [a for a in typing.get_args(ann) if a is not type(None)]
        if len(args) == 1:
            return args[0]
    return ann


def _param_type(ann) -> str:
    ann = _strip_optional(ann)
    if ann is inspect.Parameter.empty or ann is None:
        return "STRING"
    origin = typing.get_origin(ann) or ann
    if origin in PARAMETER_TYPES:
        return PARAMETER_TYPES[origin]
    if isinstance(ann, str):
        return {"str": "STRING", "int": "INT", "float": "DOUBLE", "bool": "STRING"}.get(ann, "STRING")
    return "STRING"


def _extract_interface(func: Callable):
    sig = inspect.signature(func)
    hints = {}
    for pname, ann in list(func.__annotations__.items()):
        if isinstance(ann, str):  # ``from __future__ import annotations`` in the user module
            try:
                ann = eval(ann, getattr(func, "__globals__", {}))  # noqa: S307 - user's own source
            except Exception:
                pass
        hints[pname] = ann
    inputs: List[IOSpec] = []
    outputs: List[IOSpec] = []
    for p in sig.parameters.values():
        ann = hints.get(p.name, p.annotation)
        if isinstance(ann, T.InputPath):
            inputs.append(IOSpec(io_name_for_path_arg(p.name), p.name, "artifact",
                                 T.schema_for(ann.artifact_type), "path", p.default))
        elif isinstance(ann, T.OutputPath):
            outputs.append(IOSpec(io_name_for_path_arg(p.name), p.name, "artifact",
                                  T.schema_for(ann.artifact_type), "path"))
        elif isinstance(ann, T._InputAnnotation):
            inputs.append(IOSpec(p.name, p.name, "artifact", T.schema_for(ann.artifact_type),
                                 "object", p.default))
        elif isinstance(ann, T._OutputAnnotation):
            outputs.append(IOSpec(p.name, p.name, "artifact", T.schema_for(ann.artifact_type),
                                  "object"))
        else:
            inputs.append(IOSpec(p.name, p.name, "parameter", _param_type(ann), "value",
                                 p.default, _strip_optional(ann)))
    ret = hints.get("return", sig.return_annotation)
    if ret not in (inspect.Signature.empty, None, type(None)):
        fields = getattr(ret, "_fields", None)
        if fields:  # NamedTuple
            ftypes = getattr(ret, "__annotations__", {})
            for f in fields:
                ft = ftypes.get(f)
                if isinstance(ft, type) and issubclass(ft, T.Artifact):
                    outputs.append(IOSpec(f, "", "artifact", ft.schema_title, "return"))
                else:
                    outputs.append(IOSpec(f, "", "parameter", _param_type(ft), "return",
                                          py_type=ft))
        else:
            outputs.append(IOSpec("Output", "", "parameter", _param_type(ret), "return",
                                  py_type=ret))
    names = [s.name for s in inputs + outputs]
    dup = {n for n in names if names.count(n) > 1}
    if dup:
        raise ValueError(f"component {func.__name__}: duplicate input/output names {sorted(dup)}")
    return inputs, outputs


def _function_source(func: Callable) -> str:
    try:
        src = textwrap.dedent(inspect.getsource(func))
    except (OSError, TypeError):
        # No source file (REPL / stdin / exec): ship the function by value instead.
        import base64
        import cloudpickle
        blob = base64.b64encode(cloudpickle.dumps(func)).decode("ascii")
        return (f"import base64 as _b64, cloudpickle as _cp\n"
                f"{func.__name__} = _cp.loads(_b64.b64decode({blob!r}))\n")
    lines = src.splitlines()
    # drop decorator lines (possibly multi-line) before the ``def``
    i = 0
    while i < len(lines) and not lines[i].lstrip().startswith("def "):
        i += 1
    return "\n".join(lines[i:]) + "\n"


COMPONENT_PRELUDE = (
    "import json\n"
    "from typing import *\n"
    "from mipipe.dsl import *\n"
    "from mipipe.dsl.types import *\n\n"
)


class Component:
    """A compiled-on-demand lightweight component.  Call it inside a pipeline."""

    def __init__(self, func: Callable, base_image: Optional[str] = None,
                 packages_to_install: Optional[List[str]] = None,
                 pip_index_urls: Optional[List[str]] = None):
        self.python_func = func
        self.function_name = func.__name__
        self.name = sanitize_name(func.__name__)
        self.description = inspect.getdoc(func) or ""
        self.base_image = base_image or DEFAULT_BASE_IMAGE
        self.packages_to_install = list(packages_to_install or [])
        self.pip_index_urls = list(pip_index_urls or [])
        self.inputs, self.outputs = _extract_interface(func)
        self.source = COMPONENT_PRELUDE + _function_source(func)
        self.__doc__ = func.__doc__
        self.__name__ = func.__name__
        self.__wrapped__ = func

    # ------------------------------------------------------------------ pipeline use
    def __call__(self, *args, **kwargs):
        from .pipeline import PipelineTask, current_builder
        builder = current_builder()
        if builder is None:
            raise RuntimeError(
                f"component '{self.name}' was called outside a @pipeline function. "
                "Use .python_func(...) to run the body directly.")
        bound = self._bind(args, kwargs)
        return PipelineTask(self, bound, builder)

    def _bind(self, args, kwargs) -> Dict[str, Any]:
        in_specs = self.inputs
        if len(args) > len(in_specs):
            raise TypeError(f"{self.name}() takes {len(in_specs)} inputs, got {len(args)}")
        bound: Dict[str, Any] = {}
        for spec, a in zip(in_specs, args):
            bound[spec.name] = a
        by_py = {s.py_name: s for s in in_specs}
        by_ir = {s.name: s for s in in_specs}
        for k, v in kwargs.items():
            spec = by_py.get(k) or by_ir.get(k)
            if spec is None:
                raise TypeError(f"{self.name}() got an unexpected argument {k!r}")
            if spec.name in bound:
                raise TypeError(f"{self.name}() got multiple values for {k!r}")
            bound[spec.name] = v
        for spec in in_specs:
            if spec.name not in bound and not spec.optional:
                raise TypeError(f"{self.name}() missing required input {spec.py_name!r}")
        return bound

    # ------------------------------------------------------------------ IR pieces
    def input_spec(self, name: str) -> IOSpec:
        for s in self.inputs:
            if s.name == name:
                return s
        raise KeyError(name)

    def output_spec(self, name: str) -> IOSpec:
        for s in self.outputs:
            if s.name == name:
                return s
        raise KeyError(name)

    def container_spec(self) -> Dict[str, Any]:
        """Executor container spec, kfp v2 shape: the ``sh -c`` stage installs
        ``packages_to_install`` (guarded — the MI355X node is offline, so the local
        orchestrator skips it unless MIPIPE_PIP_INSTALL=1), the ``sh -ec`` stage writes the
        inline source to a temp module and runs the executor on it."""
        pkgs = " ".join(json.dumps(p) for p in self.packages_to_install)
        install = (
            'if [ "${MIPIPE_PIP_INSTALL:-0}" = "1" ] && [ -n "' + pkgs.replace('"', "'") + '" ]; then '
            "PIP_DISABLE_PIP_VERSION_CHECK=1 python3 -m pip install --quiet --no-warn-script-location "
            + pkgs + "; fi && \"$0\" \"$@\"\n")
        program = ('program_path=$(mktemp -d)\n'
                   'printf "%s" "$0" > "$program_path/ephemeral_component.py"\n'
                   'python3 -m mipipe.dsl.executor_main '
                   '--component_module_path "$program_path/ephemeral_component.py" "$@"\n')
        return {
            "image": self.base_image,
            "command": ["sh", "-c", install, "sh", "-ec", program, self.source],
            "args": ["--executor_input", "{{$}}", "--function_to_execute", self.function_name],
        }

    def __repr__(self) -> str:
        return f"Component({self.name!r})"


def component(func: Optional[Callable] = None, *, base_image: Optional[str] = None,
              packages_to_install: Optional[List[str]] = None,
              pip_index_urls: Optional[List[str]] = None,
              output_component_file: Optional[str] = None,
              install_kfp_package: bool = True, kfp_package_path: Optional[str] = None):
    """Decorator: ``@component`` or ``@component(packages_to_install=[...])``."""

    def wrap(f):
        c = Component(f, base_image=base_image, packages_to_install=packages_to_install,
                      pip_index_urls=pip_index_urls)
        if output_component_file:
            from mipipe.compiler.compiler import component_to_yaml
            with open(output_component_file, "w") as fh:
                fh.write(component_to_yaml(c))
        return c

    if func is not None:
        return wrap(func)
    return wrap
